cd /root/repo && mkdir -p gpurun_out && timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_fullsize_golden.py -k "shard or rank or configs2" -q --timeout 300 --timeout-method thread > gpurun_out/shard_tests.log 2>&1 && timeout -k 10 300 python -u tools/shard_timing.py 64 8 > gpurun_out/shard_timing_r4b.json 2> gpurun_out/shard_timing_r4b.err; tail -3 gpurun_out/shard_tests.log; python -c "
import json
d=json.load(open('gpurun_out/shard_timing_r4b.json'))
print(d['max_rank_device_ms'], d['one_gpu_k_chain_ms'])
for r in d['per_rank']: print(r['rank'], r['device_ms'], r['k_level_ms'], r['k_chain_ms'], r['kernels'].get('k_finalize'), r['prep_ms'])
"
