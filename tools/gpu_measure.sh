#!/bin/bash
# GPU-box measurement pass: configs[2] at N=1, the sweep, per-rank shard timing
# (8 and 4 ranks in one process), chain-engine phase stamps.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-m}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload sharded --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/bench64_$TAG.json 2> gpurun_out/bench64_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload sweep --steps 5 --warmup 1 > gpurun_out/sweep_$TAG.json 2> gpurun_out/sweep_$TAG.err &&
timeout -k 10 300 python -u tools/shard_timing.py 64 8 > gpurun_out/shard8_$TAG.json 2>&1 &&
timeout -k 10 300 python -u tools/shard_timing.py 64 4 > gpurun_out/shard4_$TAG.json 2>&1 &&
GNOC_LIB=$PWD/graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python -u tools/chain_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1
rc=$?
for f in bench64 sweep shard8 shard4; do tail -n 2 gpurun_out/${f}_$TAG.json | cut -c1-600; done
cat gpurun_out/stamps_$TAG.txt | tail -40
exit $rc
