#!/bin/bash
# GPU-box: the bench with the windows each run settles on (per phase), plus the
# first run's, at a few fill targets.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for w in 2 4; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup $w --cpu-baseline 0 > gpurun_out/bw$w.json 2>gpurun_out/bw$w.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bw$w.json')); print('warmup $w', round(d['ms_per_step'],3), round(d['value']/1e9,2), d['kernel_ms']['k_chain'], d['config']['windows'], d['config']['window_ps'], d['reruns'], round(d['roofline']['frac'],4))"
done
