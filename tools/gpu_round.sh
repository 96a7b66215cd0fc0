#!/bin/bash
# One GPU-box pass: parity tests, bench, kernel-trace profile.  Every GPU step
# has its own time limit; steps are chained so the first failure ends the run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_prof_$TAG.json 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
cat gpurun_out/bench_$TAG.json
exit $rc
