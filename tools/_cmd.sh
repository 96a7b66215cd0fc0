mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r2a.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_r2a.log; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_r2a.log | awk '{print $NF}' | sort | uniq -c
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/chain_check.py > gpurun_out/cc_r2a.log 2>&1; echo cc rc=$?; tail -1 gpurun_out/cc_r2a.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_r2a.json 2> gpurun_out/bench_r2a.err; echo bench rc=$?
cat gpurun_out/bench_r2a.json
