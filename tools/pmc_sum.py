#!/usr/bin/env python3
"""Mean per launch of every counter in rocprofv3 --pmc output directories, per
kernel (name filter optional): python tools/pmc_sum.py DIR [DIR ...] [-k k_chain]"""
import csv
import glob
import os
import sys
from collections import defaultdict

args = sys.argv[1:]
filt = None
if "-k" in args:
    i = args.index("-k")
    filt = args[i + 1]
    del args[i:i + 2]
acc = defaultdict(lambda: defaultdict(list))
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                if filt and filt not in k:
                    continue
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
                acc[k][key].append(float(r["Counter_Value"]))
for k, m in acc.items():
    per = defaultdict(list)
    for (disp, cn), vals in m.items():
        per[cn].append(sum(vals))
    print(k)
    for cn in sorted(per):
        v = per[cn]
        print(f"  {cn:24s} launches={len(v):4d} mean={sum(v) / len(v):.4g}")
