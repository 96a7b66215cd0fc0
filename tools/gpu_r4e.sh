#!/bin/bash
# Round-4 GPU pass: M/G/1 chain tests, sweep decline reasons, bench, stamps, full suite.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r4e}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_excmerge.py tests/test_gpu_fullsize_golden.py -k "excmerge or burst or mg1" -x -q -s --timeout 120 --timeout-method thread > gpurun_out/pytest_mg_$TAG.log 2>&1 &&
GNOC_CHAIN_DEBUG=1 timeout -k 10 300 python -u bench.py --workload sweep --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/sweepdbg_$TAG.json 2> gpurun_out/sweepdbg_$TAG.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
GNOC_LIB=$PWD/graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python -u tools/chain_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_mg_$TAG.log
grep "declined" gpurun_out/sweepdbg_$TAG.err | sort | uniq -c | head
head -c 300 gpurun_out/sweepdbg_$TAG.json; echo
head -c 400 gpurun_out/bench_$TAG.json; echo
grep -E "phase|land|wait|emit|step  |span|utilis" gpurun_out/stamps_$TAG.txt
tail -3 gpurun_out/pytest_$TAG.log
exit $rc
