cd /root/repo
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_full.log | tail -8
grep -E "^E " gpurun_out/pytest_full.log | head -5
exit $rc
