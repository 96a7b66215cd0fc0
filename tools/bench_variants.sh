#!/bin/bash
# On the GPU box: quick bench of every variant library (no CPU baseline).
# Extra bench.py arguments pass through (e.g. --workload sharded).
cd "$(dirname "$0")/.." || exit 1
for so in graphite_amd/_build/var/*.so; do
  n=$(basename $so .so)
  GNOC_LIB=$PWD/$so timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 "$@" > gpurun_out/var_${n}${VTAG}.json 2>/dev/null || { echo "$n FAILED"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var_${n}${VTAG}.json')); print('$n', round(d['value']/1e9,2), 'G hops/s', round(d['ms_per_step'],2), 'ms', 'k_level', d['kernel_ms']['k_level'])"
done
