#!/bin/bash
# A/B timing of libgnoc variants on configs[1]: tools/gpu_ab.sh OUT name1 name2 ... (name "cur" = libgnoc.so),
# each run twice, interleaved; extra env via AB_HOT (hotspot fraction).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/$1; shift
: > $out
for rep in 1 2; do
  for v in "$@"; do
    lib=graphite_amd/_build/libgnoc.so; [ "$v" != cur ] && lib=graphite_amd/_build/libgnoc_$v.so
    GNOC_LIB=$lib timeout -k 10 120 python -u tools/run_probe.py 10 ${AB_HOT:-0} >> $out 2>&1 || { tail -5 $out; exit 1; }
  done
done
grep "^lib" $out
