#!/bin/bash
# Round-4 GPU pass: M/G/1 chain tests first, then everything, bench (mesh + sweep), stamps,
# then the bench on the DPP-rank build (libgnoc_nobrank.so, CH_BRANK=0) for comparison.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
TAG=${1:-r4d}
V=$PWD/graphite_amd/_build/libgnoc_nobrank.so
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_excmerge.py tests/test_gpu_fullsize_golden.py -k "excmerge or burst or mg1" -x -q -s --timeout 120 --timeout-method thread > gpurun_out/pytest_mg_$TAG.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u bench.py --workload sweep --steps 5 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_sweep_$TAG.json 2> gpurun_out/bench_sweep_$TAG.err &&
GNOC_LIB=$PWD/graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python -u tools/chain_stamps.py > gpurun_out/stamps_$TAG.txt 2>&1 &&
GNOC_LIB=$V timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/bench_brank_$TAG.json 2> gpurun_out/bench_brank_$TAG.err
rc=$?
tail -5 gpurun_out/pytest_mg_$TAG.log
tail -3 gpurun_out/pytest_$TAG.log
head -c 700 gpurun_out/bench_$TAG.json; echo
head -c 700 gpurun_out/bench_sweep_$TAG.json; echo
grep -E "phase|land|step  |span|utilis" gpurun_out/stamps_$TAG.txt
head -c 700 gpurun_out/bench_brank_$TAG.json; echo
exit $rc
