mkdir -p gpurun_out
for L in libgnoc_64a.so libgnoc_64b.so libgnoc_128.so libgnoc.so; do
  GNOC_LIB=$PWD/graphite_amd/_build/$L timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 > gpurun_out/b_$L.json 2> gpurun_out/b_$L.err || { tail -5 gpurun_out/b_$L.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/b_$L.json')); k=d['kernel_ms']; print('$L', round(d['value']/1e9,2), 'G hops/s', round(d['ms_per_step'],3), 'ms chain', k['k_chain'], 'level', k['k_level'])"
done
GNOC_LIB=$PWD/graphite_amd/_build/libgnoc_64a.so timeout -k 10 300 python -u tools/chain_check.py > gpurun_out/cc7.log 2>&1; tail -4 gpurun_out/cc7.log
