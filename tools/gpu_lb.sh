#!/bin/bash
# GPU-box: look-back chain engine: quick parity, then bench of the default and a variant lib.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
P=gpurun_out/lb_${1:-a}
mkdir -p $P
GNOC_CHAIN_DEBUG=1 timeout -k 10 240 python3 -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_parity.py -k "synthetic_8x8 or uniform_32x32 or hotspot_32x32 or mesh_shapes or frequency_chain or saturated or declined" > $P/pytest.log 2>&1
rc=$?; tail -4 $P/pytest.log; grep -c "declined" $P/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in ${LIBS:-libgnoc.so}; do
  GNOC_LIB=graphite_amd/_build/$L GNOC_CHAIN_DEBUG=1 timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 > $P/b_$L.json 2> $P/b_$L.err
  rc=$?; python3 tools/bench_line.py $P/b_$L.json $L; grep -m3 "declined" $P/b_$L.err; [ $rc -eq 0 ] || exit $rc
done
