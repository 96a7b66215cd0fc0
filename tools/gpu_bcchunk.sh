#!/bin/bash
# k_level chunk targets for the full-level runs: broadcast batches, the level engine on
# configs[1], the 256-point sweep.  tools/gpu_bcchunk.sh CHUNK ...
export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/r6_bcchunk2.log
for ch in "$@"; do
  echo "chunk $ch" >> gpurun_out/r6_bcchunk2.log
  GNOC_CHUNK=$ch timeout -k 10 200 python -u tools/bcast_timing.py 32 10000 1e-4 >> gpurun_out/r6_bcchunk2.log 2>&1 || exit 1
  GNOC_ENGINE=levels GNOC_CHUNK=$ch timeout -k 10 100 python -u tools/run_probe.py 6 >> gpurun_out/r6_bcchunk2.log 2>&1 || exit 1
  GNOC_CHUNK=$ch timeout -k 10 200 python -u bench.py --workload sweep --steps 5 --warmup 1 --cpu-baseline 0 > gpurun_out/r6_sw_$ch.json 2>&1 || exit 1
  python3 -c "import json,sys; [print('sweep', json.loads(l)['ms_per_step'], json.loads(l)['config'].get('engine_path')) for l in open('gpurun_out/r6_sw_$ch.json') if l.startswith('{')]" >> gpurun_out/r6_bcchunk2.log
done
grep -v amdgpu gpurun_out/r6_bcchunk2.log
