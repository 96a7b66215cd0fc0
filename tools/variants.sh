#!/bin/bash
# Build libgnoc variants (extra -D flags) into graphite_amd/_build/var/<name>.so
# usage: tools/variants.sh name "-DFOO=1" [name2 "-D..."]...
cd "$(dirname "$0")/.." || exit 1
mkdir -p graphite_amd/_build/var
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Iinclude -Igraphite_amd/csrc $2 \
     -o graphite_amd/_build/var/$1.so graphite_amd/csrc/engine.hip graphite_amd/csrc/trace.cpp -L/opt/rocm/lib -lrccl &
  shift 2
done
wait
