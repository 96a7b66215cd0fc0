#!/bin/bash
# GPU-box: bench line (configs[1] uniform + hotspot) of each library named on the
# command line (paths relative to graphite_amd/_build/); one digest line each.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/var
for v in "$@"; do
  n=$(basename $v .so)
  GNOC_LIB=graphite_amd/_build/$v timeout -k 10 150 python3 -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/var/$n.json 2> gpurun_out/var/$n.err
  rc=$?
  python3 tools/bench_line.py gpurun_out/var/$n.json $n || tail -3 gpurun_out/var/$n.err
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
done
exit 0
