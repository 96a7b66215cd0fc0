cd /root/repo
export TMPDIR=/tmp
VTAG=_32 bash tools/bench_variants.sh && VTAG=_64 bash tools/bench_variants.sh --workload sharded &&
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r4.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_r4.log
exit $rc
