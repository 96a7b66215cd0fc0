#!/bin/bash
# One GPU-box pass: parity tests, bench, kernel-trace profile, then the two
# PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass: 3 + 2 TCC slots).
# Every GPU step has its own time limit; steps are chained so the first failure
# ends the run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r1}
P=gpurun_out/prof_$TAG
mkdir -p $P ${P}_hot
BENCH="bench.py --steps 10 --warmup 2 --cpu-baseline 0 --hotspot 0 --e2e 0"   # the first run sizes the chain windows: a small share of the average
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $P -o run -- python3 -u $BENCH > $P/bench_kt.json 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d ${P}_hot -o run -- python3 -u $BENCH --mix hotspot > ${P}_hot/bench_kt.json 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P -o fetch -- python3 -u $BENCH > $P/bench_fetch.json 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P -o write -- python3 -u $BENCH > $P/bench_write.json 2>&1 &&
python3 tools/prof_summary.py $P > $P/summary.txt && python3 tools/prof_summary.py ${P}_hot > ${P}_hot_summary.txt
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
cat gpurun_out/bench_$TAG.json
cat $P/summary.txt 2>/dev/null
exit $rc
