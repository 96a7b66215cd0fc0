#!/bin/bash
# GPU-box pass: selected tests (pytest -k EXPR) then the moving-average timings.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-q}; K=${2:-moving_average}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 120 python -u tools/ma_timing.py 10000 1 64 > gpurun_out/ma1_$TAG.txt 2>&1 &&
timeout -k 10 120 python -u tools/ma_timing.py 10000 2 64 > gpurun_out/ma2_$TAG.txt 2>&1 &&
timeout -k 10 120 python -u tools/ma_timing.py 10000 3 64 > gpurun_out/ma3_$TAG.txt 2>&1
rc=$?
tail -n 15 gpurun_out/pytest_$TAG.log
for f in gpurun_out/ma1_$TAG.txt gpurun_out/ma2_$TAG.txt gpurun_out/ma3_$TAG.txt; do tail -n 1 $f; done
exit $rc
