#!/bin/bash
# GPU-box: bench the chain-engine build variants (graphite_amd/_build/var/*.so)
# and window fills; one line per run: variant fill ms_per_step k_chain windows reruns.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/variants_${1:-v}.txt
: > $OUT
run() {  # lib fill
  GNOC_LIB=$1 GNOC_CH_FILL=$2 timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --cpu-baseline 0 > gpurun_out/vb.json 2>/dev/null
  rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/vb.json')); print(sys.argv[1].split('/')[-1], sys.argv[2], round(d['ms_per_step'],3), d['kernel_ms']['k_chain'], d['config']['windows'], d['reruns'], d['config']['engine_path'])" $1 $2 >> $OUT 2>&1 || echo "$1 $2 rc=$rc" >> $OUT
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && return 1
  return 0
}
B=$PWD/graphite_amd/_build
run $B/libgnoc.so 0.55 && run $B/libgnoc.so 1.2 &&
for v in per9 per10 per12 minw4; do run $B/var/$v.so 0.55 || break; done
cat $OUT
