mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_validate.py tests/test_host_cpp.py tests/test_abi.py tests/test_gpu_patterns.py tests/test_gpu_proxy.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_new.log | sed 's/.*:://' | cut -c1-110; tail -3 gpurun_out/pytest_new.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline 0 > gpurun_out/bench_val.json 2> gpurun_out/bench_val.err; echo bench rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/bench_val.json')); print(d['value']/1e9, d['ms_per_step'], d['e2e_ms_per_step'], d['kernel_ms']['k_chain'])"
