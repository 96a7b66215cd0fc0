#!/bin/bash
# 8-rank 64x64 shard timing on one GPU under environment variants: tools/gpu_shard_ab.sh "VAR=VAL ..." ...
export TMPDIR=/tmp; mkdir -p gpurun_out; : > gpurun_out/shard_ab.log
for v in "$@"; do
  echo "variant $v" >> gpurun_out/shard_ab.log
  env $v timeout -k 10 200 python -u tools/shard_timing.py 64 8 > gpurun_out/shard_ab_tmp.json 2>> gpurun_out/shard_ab.log || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/shard_ab_tmp.json'))
print('busiest', d['max_rank_device_ms'], 'one-gpu chain', d['one_gpu_k_chain_ms'], 'chain per rank', [r['k_chain_ms'] for r in d['per_rank']])" >> gpurun_out/shard_ab.log
done
grep -v amdgpu gpurun_out/shard_ab.log
