#!/bin/bash
# Round-6 secondary measurements on the committed build: configs[2] on one GPU, the
# 256-point sweep, the 8-rank 64x64 rehearsal on one GPU, broadcast passes.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --mesh 64 --steps 5 --warmup 1 --cpu-baseline 0 --hotspot 0 --e2e 0 > gpurun_out/r6x_64.json 2> gpurun_out/r6x_64.err &&
timeout -k 10 300 python -u bench.py --workload sweep --steps 5 --warmup 1 --cpu-baseline 0 > gpurun_out/r6x_sweep.json 2> gpurun_out/r6x_sweep.err &&
timeout -k 10 300 python -u tools/shard_timing.py 64 8 > gpurun_out/r6x_shard8.json 2> gpurun_out/r6x_shard8.err &&
GNOC_BCAST_DEBUG=1 timeout -k 10 300 python -u tools/bcast_timing.py 32 10000 1e-4 3e-4 > gpurun_out/r6x_bcast.txt 2>&1
rc=$?
grep -h '^{' gpurun_out/r6x_64.json gpurun_out/r6x_sweep.json | cut -c1-300
grep "W=32" gpurun_out/r6x_bcast.txt
exit $rc
