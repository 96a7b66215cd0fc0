#!/bin/bash
# Build a libgnoc variant with chain-engine tile macros: tools/build_variant.sh NAME -DCH_T_V=... ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Iinclude -Igraphite_amd/csrc \
  "$@" -o graphite_amd/_build/libgnoc_$name.so graphite_amd/csrc/engine.hip graphite_amd/csrc/trace.cpp -L/opt/rocm/lib -lrccl
