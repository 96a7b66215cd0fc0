cd /tmp && export TMPDIR=/tmp && cd /root/repo && mkdir -p gpurun_out/kt_shard && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_shard -o kt -- python3 -u tools/shard_timing.py 64 8 > gpurun_out/kt_shard/out.json 2>&1; python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/kt_shard/**/kt_kernel_trace.csv', recursive=True) or glob.glob('gpurun_out/kt_shard/*kernel_trace.csv')
rows = list(csv.DictReader(open(f[0])))
lv = [r for r in rows if 'k_level' in r['Kernel_Name']]
print(len(lv), 'k_level dispatches')
for r in lv[-40:]:
    print(r['Grid_Size'], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000.0)
PY
