#!/bin/bash
# Round-6 GPU pass G: parity suite (sample-searched window bounds), A/B of the number of
# variable-window adaptations, per-kernel times.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6g_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r6g_pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r6g_ab.log cur cur+GNOC_CH_ADAPT_RUNS=8 cur+GNOC_CH_VARWIN=0 || exit 1
AB_HOT=0.2 bash tools/gpu_ab.sh r6g_ab_hot.log cur cur+GNOC_CH_ADAPT_RUNS=8 cur+GNOC_CH_VARWIN=0 || exit 1
GNOC_PROBE_PROF=1 timeout -k 10 120 python -u tools/run_probe.py 10 > gpurun_out/r6g_prof.log 2>&1
rc=$?
cat gpurun_out/r6g_prof.log
exit $rc
