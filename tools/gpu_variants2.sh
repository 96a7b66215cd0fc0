#!/bin/bash
# GPU-box: bench of the build variants in graphite_amd/_build/var (adapted windows settle in the warmup).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for lib in $PWD/graphite_amd/_build/libgnoc.so $PWD/graphite_amd/_build/var/*.so; do
  GNOC_LIB=$lib timeout -k 10 150 python -u bench.py --steps 5 --warmup 3 --cpu-baseline 0 > gpurun_out/vb.json 2>/dev/null || { echo "$lib failed"; continue; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/vb.json')); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],3), d['kernel_ms']['k_chain'], d['config']['windows'], d['reruns'])" $lib
done
