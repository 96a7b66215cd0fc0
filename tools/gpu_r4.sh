#!/bin/bash
# Round-4 GPU pass: parity tests, bench, separate-launch stamps, fused-launch timing.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r4}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
GNOC_LIB=$PWD/graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python -u tools/chain_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 &&
GNOC_XY=1 timeout -k 10 300 python -u tools/xy_lag.py 0.6,1.0 > gpurun_out/xylag_$TAG.txt 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
head -c 600 gpurun_out/bench_$TAG.json; echo
grep -E "phase|land|step  |span|utilis" gpurun_out/stamps_$TAG.txt
cat gpurun_out/xylag_$TAG.txt
exit $rc
