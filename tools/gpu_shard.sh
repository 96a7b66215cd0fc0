#!/bin/bash
# GPU-box pass for the sharded path: shard tests, then the regular GPU suite.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-sh}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "SHARD|passed|failed|Error|error" gpurun_out/pytest_$TAG.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}_all.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_${TAG}_all.log
exit $rc
