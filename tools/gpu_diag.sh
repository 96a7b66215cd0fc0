#!/bin/bash
# GPU-box diagnosis pass: chosen parity tests, chain stamps (uniform + hotspot) on
# the -DCH_STAMPS build, SQ counters of the bench.  First failure ends the run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-d}
P=gpurun_out/diag_$TAG
mkdir -p $P
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py} > $P/pytest.log 2>&1
rc=$?; tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python3 -u tools/chain_stamps.py > $P/stamps_uniform.txt 2>&1 &&
GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python3 -u tools/chain_stamps.py 32 0.005 10000 hotspot > $P/stamps_hotspot.txt 2>&1 &&
bash tools/gpu_sq.sh $TAG > /dev/null 2>&1
rc=$?
cat $P/stamps_uniform.txt | grep -v amdgpu.ids; cat gpurun_out/sq_$TAG/sum.txt 2>/dev/null | head -40
exit $rc
