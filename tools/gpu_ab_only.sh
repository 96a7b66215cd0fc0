#!/bin/bash
# A/B of libgnoc variants only (no parity suite): uniform then hotspot.  tools/gpu_ab_only.sh TAG VARIANT ...
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
bash tools/gpu_ab.sh ${TAG}_ab.log "$@" || exit 1
AB_HOT=0.2 bash tools/gpu_ab.sh ${TAG}_ab_hot.log "$@"
