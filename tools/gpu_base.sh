#!/bin/bash
# GPU-box: configs[1] uniform + hotspot bench lines and a kernel-trace profile of each
# (the same-HEAD evidence the bench's roofline is recomputed from).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-base}
P=gpurun_out/base_$TAG
mkdir -p $P
git_head=$(cat .git_head 2>/dev/null || echo unknown)
echo "head $git_head" > $P/head.txt
B="bench.py --steps 10 --warmup 3 --cpu-baseline 0"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > $P/uniform.json 2> $P/uniform.err &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 --mix hotspot > $P/hotspot.json 2> $P/hotspot.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $P/ku -o run -- python3 -u $B > $P/ku.json 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kh -o run -- python3 -u $B --mix hotspot > $P/kh.json 2>&1 &&
python3 tools/prof_summary.py $P/ku > $P/ku_summary.txt && python3 tools/prof_summary.py $P/kh > $P/kh_summary.txt
rc=$?
head -5 $P/ku_summary.txt $P/kh_summary.txt
exit $rc
