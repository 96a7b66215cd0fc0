#!/bin/bash
# Round-6 GPU pass D: parity suite with variable chain windows, A/B against uniform
# windows per chain (uniform and hotspot traffic), per-kernel times.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r6d_pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r6d_ab.log cur cur+GNOC_CH_VARWIN=0 || exit 1
AB_HOT=0.2 bash tools/gpu_ab.sh r6d_ab_hot.log cur cur+GNOC_CH_VARWIN=0 || exit 1
GNOC_PROBE_PROF=1 timeout -k 10 120 python -u tools/run_probe.py 10 > gpurun_out/r6d_prof.log 2>&1
rc=$?
cat gpurun_out/r6d_prof.log
exit $rc
