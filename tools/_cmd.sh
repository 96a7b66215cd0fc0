cd /root/repo
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_t.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_t.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value']/1e9, d['ms_per_step'], d['kernel_ms'])" || exit 1; done
