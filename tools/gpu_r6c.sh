#!/bin/bash
# Round-6 GPU pass C: parity suite with XCD-local chain queues on, A/B against the one
# shared queue (uniform and hotspot), and the stamps of the XCD-local build.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6c_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r6c_pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh r6c_ab.log cur cur+GNOC_CH_XCD=0 || exit 1
AB_HOT=0.2 bash tools/gpu_ab.sh r6c_ab_hot.log cur cur+GNOC_CH_XCD=0 || exit 1
GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so CH_STAMPS_DUMP=gpurun_out/r6c_st timeout -k 10 200 python3 -u tools/chain_stamps.py > gpurun_out/r6c_stamps.txt 2>&1
rc=$?
grep "phase\|step  \|wait\|utilisation\|span" gpurun_out/r6c_stamps.txt
exit $rc
