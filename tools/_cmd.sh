mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_host_cpp.py tests/test_abi.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_cshard.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_cshard.log | sed 's/.*:://' | cut -c1-110 | tail -8; tail -25 gpurun_out/pytest_cshard.log | grep -v PASSED | head -20; exit $rc
