#!/bin/bash
# GPU pass: parity suite, then A/B of libgnoc variants (tools/gpu_ab.sh) on uniform and
# hotspot traffic, then per-kernel times.  tools/gpu_check.sh TAG VARIANT ...
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh ${TAG}_ab.log "$@" || exit 1
AB_HOT=0.2 bash tools/gpu_ab.sh ${TAG}_ab_hot.log "$@" || exit 1
GNOC_PROBE_PROF=1 timeout -k 10 120 python -u tools/run_probe.py 10 > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
cat gpurun_out/${TAG}_prof.log
exit $rc
