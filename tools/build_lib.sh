#!/bin/bash
# Rebuild only libgnoc.so (the HIP engine + C ABI), as __graft_entry__.build() does.
cd "$(dirname "$0")/.." || exit 1
python3 -c "
import __graft_entry__ as g, os
out = os.path.join(g.ROOT, 'graphite_amd', '_build')
g._run([g.HIPCC, f'--offload-arch={g.ARCH}'] + g.LIB_FLAGS + [f'-DGNOC_BUILD_ID=\"{g.build_id()}\"', '-Iinclude',
       '-Igraphite_amd/csrc', '-o', os.path.join(out, 'libgnoc.so')] + g.LIB_SOURCES + ['-L/opt/rocm/lib', '-lrccl'])
"
