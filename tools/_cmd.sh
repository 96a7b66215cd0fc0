cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sweep.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload sweep --steps 3 --warmup 1 > gpurun_out/b_sweep.json 2> gpurun_out/b_sweep.err
rc=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_sweep.log | tail -6
tail -2 gpurun_out/pytest_all.log
grep -E "^FAILED|^E " gpurun_out/pytest_all.log | head -5
cat gpurun_out/b_sweep.json; tail -3 gpurun_out/b_sweep.err
exit $rc
