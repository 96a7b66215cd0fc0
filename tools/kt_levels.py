"""Per-kernel mean durations (us) from a rocprofv3 kernel trace directory, the
k_level launches split by their order within a run (first = injection level,
last = SELF level on the chain path).

    python tools/kt_levels.py DIR
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = defaultdict(list)
    lv = 0
    for r in rows:
        nm = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        if nm == "k_classify":
            lv = 0
        if nm == "k_level":
            nm = f"k_level#{lv}"
            lv += 1
        d[nm].append(us)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v2 = v[2:] if len(v) > 4 else v
        print(f"{k:28s} n={len(v):4d} mean(after 2) {sum(v2) / len(v2):9.1f} us")


if __name__ == "__main__":
    main()
