#!/bin/bash
# Round-6 GPU pass B: A/B of chain variants, and a stamps build's raw per-step stamps.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh r6b_ab.log cur tp rktp || exit 1
GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so CH_STAMPS_DUMP=gpurun_out/r6b_st timeout -k 10 200 python3 -u tools/chain_stamps.py > gpurun_out/r6b_stamps.txt 2>&1
rc=$?
tail -5 gpurun_out/r6b_stamps.txt
exit $rc
