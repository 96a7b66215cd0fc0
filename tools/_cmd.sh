cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_virgin.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_virgin.log
grep -E "^FAILED|^E " gpurun_out/pytest_virgin.log | head
exit $rc
