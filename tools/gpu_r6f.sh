#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh r6f_ab.log cur cur+GNOC_CH_TARGET_V=0.92 cur+GNOC_CH_TARGET_V=0.78 cur+GNOC_CH_VARWIN=0 || exit 1
AB_HOT=0.2 bash tools/gpu_ab.sh r6f_ab_hot.log cur cur+GNOC_CH_TARGET_V=0.92 cur+GNOC_CH_TARGET_V=0.78 cur+GNOC_CH_VARWIN=0 || exit 1
