cd /root/repo
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_sc.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload sweep --steps 3 --warmup 1 > gpurun_out/b_sweep.json 2>/dev/null
rc=$?
tail -2 gpurun_out/pytest_sc.log
python3 -c "
import json
for f in ['b_sweep']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, round(d['value']/1e9,2), round(d['ms_per_step'],3), {k:v for k,v in d['kernel_ms'].items() if v>0.05})
"
exit $rc
