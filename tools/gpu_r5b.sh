#!/bin/bash
# Round-5 GPU pass: full GPU suite, wave-priority variant timing, staged scatter
# parity (configs[1] SHA pins) and kernel-trace timing.  Every GPU step has its
# own limit; the first failure ends the run.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipe.py tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_r5b.log 2>&1 || { tail -30 $O/pytest_r5b.log; exit 1; }
tail -3 $O/pytest_r5b.log
for v in cur prio2 cur prio2; do
  lib=graphite_amd/_build/libgnoc.so; [ $v = prio2 ] && lib=graphite_amd/_build/libgnoc_prio2.so
  GNOC_LIB=$lib timeout -k 10 120 python -u tools/run_probe.py 10 >> $O/prio.log 2>&1 || exit 1
done
cat $O/prio.log
GNOC_SCATTER_STAGE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize_golden.py -x -q --timeout 300 --timeout-method thread -k "configs1_full_size_matches" > $O/pytest_st.log 2>&1 || { tail -30 $O/pytest_st.log; exit 1; }
tail -2 $O/pytest_st.log
for st in 0 1; do
  GNOC_SCATTER_STAGE=$st timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_st$st -o run -- python3 -u tools/run_probe.py 8 > $O/kt_st$st.log 2>&1 || exit 1
  python3 tools/kt_levels.py $O/kt_st$st > $O/kt_st$st.txt; head -8 $O/kt_st$st.txt
done
