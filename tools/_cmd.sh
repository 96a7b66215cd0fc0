cd /root/repo
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_t.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_t.log; [ $rc -ne 0 ] && exit $rc
bash tools/bench_variants.sh && GNOC_LIB=$PWD/graphite_amd/_build/var/lb4.so timeout -k 10 200 python -u tools/stamps.py 32 10000
