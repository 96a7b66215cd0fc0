cd /root/repo
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_hc.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_hc.log
grep -E "^FAILED|^E " gpurun_out/pytest_hc.log | head -8
exit $rc
