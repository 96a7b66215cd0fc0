#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
GNOC_CHAIN_DEBUG=1 timeout -k 10 60 python -u tools/dbg_gap.py > gpurun_out/r6e_dbg.log 2>&1 || exit 1
cat gpurun_out/r6e_dbg.log
bash tools/gpu_r6d.sh
