#!/bin/bash
# rocprofv3 kernel stats of a broadcast batch (tools/bcast_timing.py), current vs another libgnoc build
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in cur old; do
  lib=graphite_amd/_build/libgnoc.so
  [ "$v" = old ] && lib=graphite_amd/_build/libgnoc_old.so
  GNOC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof_$v -o run -- python3 -u tools/bcast_timing.py 32 10000 1e-4 > gpurun_out/bprof_$v.log 2>&1
done
