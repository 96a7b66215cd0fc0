#!/bin/bash
# GPU-box iteration: parity tests that pin the chain engine, then the bench line
# (configs[1] uniform + hotspot).  Every GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-q}
P=gpurun_out/q_$TAG
mkdir -p $P
timeout -k 10 ${TEST_TIMEOUT:-400} python3 -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_fullsize_golden.py tests/test_gpu_patterns.py} > $P/pytest.log 2>&1
rc=$?
tail -3 $P/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > $P/bench.json 2> $P/bench.err; rc=$?
python3 tools/bench_line.py $P/bench.json $TAG
exit $rc
