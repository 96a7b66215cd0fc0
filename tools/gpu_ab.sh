#!/bin/bash
# GPU-box A/B: bench of two libgnoc builds on the same box (GNOC_LIB), interleaved.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for lib in "$@"; do
  GNOC_LIB=$lib timeout -k 10 120 python -u bench.py --steps 5 --warmup 3 --cpu-baseline 0 > gpurun_out/ab.json 2>/dev/null || { echo "$lib failed"; continue; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1].split('/')[-1], round(d['ms_per_step'],3), d['kernel_ms']['k_chain'], d['config'].get('windows'), d['config'].get('window_ps'))" $lib
done
done
