#!/bin/bash
# Round-end GPU pass on the committed build: parity + bench + profiles (tools/gpu_round.sh),
# chain stamps (libgnoc_stamps.so) and SQ counters (tools/gpu_sq.sh).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r4c}
bash tools/gpu_round.sh $TAG > gpurun_out/round_$TAG.txt 2>&1 &&
GNOC_LIB=$PWD/graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python -u tools/chain_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 &&
bash tools/gpu_sq.sh $TAG > gpurun_out/sq_$TAG.txt 2>&1
rc=$?
tail -12 gpurun_out/round_$TAG.txt
grep -E "phase|span|utilis" gpurun_out/stamps_$TAG.txt
tail -40 gpurun_out/sq_$TAG.txt
exit $rc
