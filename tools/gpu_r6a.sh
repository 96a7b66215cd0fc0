#!/bin/bash
# Round-6 GPU pass A: parity suite on the cleaned-up build, an A/B of the plain-store
# turn variant, and one run of the SELF-level no-final-store variant under a kernel trace.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6a_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r6a_pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r6a_ab.log cur tp || exit 1
GNOC_LIB=graphite_amd/_build/libgnoc_nofin.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6a_nofin -o run -- python3 -u tools/run_probe.py 8 > gpurun_out/r6a_nofin.log 2>&1
rc=$?
grep "^lib" gpurun_out/r6a_nofin.log
exit $rc
