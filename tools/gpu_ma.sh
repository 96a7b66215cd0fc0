#!/bin/bash
# GPU-box pass: the whole GPU suite, moving-average timings (three averages),
# a kernel-trace profile of the arithmetic-mean run, and the bench.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-ma}
P=gpurun_out/prof_$TAG
mkdir -p $P
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 120 python -u tools/ma_timing.py 10000 1 64 > gpurun_out/ma1_$TAG.txt 2>&1 &&
timeout -k 10 120 python -u tools/ma_timing.py 10000 2 64 > gpurun_out/ma2_$TAG.txt 2>&1 &&
timeout -k 10 120 python -u tools/ma_timing.py 10000 3 64 > gpurun_out/ma3_$TAG.txt 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o ma -- python3 -u tools/ma_timing.py 10000 1 64 > $P/ma_kt.txt 2>&1 &&
timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
tail -1 gpurun_out/ma1_$TAG.txt gpurun_out/ma2_$TAG.txt gpurun_out/ma3_$TAG.txt
cat gpurun_out/bench_$TAG.json
exit $rc
