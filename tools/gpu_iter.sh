#!/bin/bash
# GPU-box iteration: the bench line (configs[1] uniform + hotspot) of a reference
# build (GNOC_LIB=$REF, default the round-2 library) and of the current build, then
# the parity tests that pin the chain engine.  Every GPU step has its own time
# limit; the first failure ends the run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-it}
REF=${REF:-graphite_amd/_build/libgnoc_r2.so}
P=gpurun_out/it_$TAG
mkdir -p $P
B="--steps 20 --warmup 3 --cpu-baseline 0"
line() { python3 tools/bench_line.py $1 $2; }
if [ -z "$NOREF" ] && [ -f "$REF" ]; then
  GNOC_LIB=$REF timeout -k 10 300 python3 -u bench.py $B > $P/ref.json 2> $P/ref.err; line $P/ref.json ref || exit 1
fi
timeout -k 10 ${TEST_TIMEOUT:-400} python3 -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_fullsize_golden.py} > $P/pytest.log 2>&1
rc=$?
tail -5 $P/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py $B > $P/new.json 2> $P/new.err; line $P/new.json new
