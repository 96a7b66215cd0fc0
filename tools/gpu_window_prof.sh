#!/bin/bash
# GPU-box: per-phase k_chain time (rocprofv3 kernel stats) at fixed X / Y window sizes.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/wprof
for xy in "8388608 8388608" "12400000 8388608" "16000000 8388608" "20000000 8388608" "8388608 9000000" "8388608 7000000"; do
  set -- $xy
  d=gpurun_out/wprof/x$1_y$2
  GNOC_WINDOW_PS_X=$1 GNOC_WINDOW_PS_Y=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o w -- python3 -u tools/window_trace.py 4 > $d.txt 2>&1 || { echo "fail $xy"; exit 1; }
  python3 - $d $1 $2 <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/w_kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
out = {}
for r in rows:
    if "k_chain" in r["Name"]:
        out["X" if "<1>" in r["Name"] else "Y"] = float(r["AverageNs"]) / 1e3
print("X", sys.argv[2], "Y", sys.argv[3], "avg us per launch:", {k: round(v, 1) for k, v in sorted(out.items())})
PY
  tail -n 1 $d.txt
done
