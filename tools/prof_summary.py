"""Summarise a tools/gpu_round.sh profile directory: per-kernel time, the
per-level k_level durations and launch gaps (kernel trace), and HBM bytes per
launch of the dominant kernel (k_chain on v4, k_level on v3) and of k_level,
from the FETCH_SIZE / WRITE_SIZE passes.  Writes pmc.json next
to the CSVs (bench.py reads the committed copy for roofline.traffic).

FETCH_SIZE is doubled per MI355X_MICROARCH.md "HBM [CDNA4]" (gfx950 tallies
128-B fabric reads at 64 B); WRITE_SIZE is taken as is."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]


def rows(pattern):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


kt = rows("run_kernel_trace.csv")
kt.sort(key=lambda r: int(r["Start_Timestamp"]))
per = defaultdict(list)
for r in kt:
    per[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print("kernel                calls   avg_us   total_ms")
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:20s} {len(v):6d} {sum(v) / len(v) / 1e3:8.2f} {sum(v) / 1e6:10.3f}")
# the profiled command's first runs size the chain windows (different windows, and a
# first run that adapts them): the steady state is the launches after those runs
STEADY = 20
for k in ("k_chain", "k_level"):
    v = per.get(k, [])
    if len(v) > STEADY:
        t = v[-STEADY:]
        print(f"{k} steady state (its last {STEADY} launches, after the window settle runs): avg_us "
              f"{sum(t) / len(t) / 1e3:.2f}, min {min(t) / 1e3:.2f}, max {max(t) / 1e3:.2f}")

# one step = the kernels from a k_classify launch to the next k_finalize; use the
# last complete step: its kernels, busy time, span and the gaps between launches
steps, cur = [], None
for r in kt:
    n = short(r["Kernel_Name"])
    if n == "k_classify":
        cur = []
    if cur is not None:
        cur.append(r)
        if n == "k_finalize":
            steps.append(cur)
            cur = None
if steps:
    last = steps[-1]
    se = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in last)
    busy = sum(e - s for s, e, _ in se)
    gaps = [max(0, se[i + 1][0] - se[i][1]) for i in range(len(se) - 1)]
    print(f"\nlast step: {len(se)} kernels, busy {busy / 1e6:.3f} ms, span {(se[-1][1] - se[0][0]) / 1e6:.3f} ms, "
          f"gaps between launches {sum(gaps) / 1e6:.3f} ms")
    print("  " + ", ".join(f"{n} {(e - s) / 1e3:.1f}" for s, e, n in se))


def pmc(pattern, counter, kernel):
    vals = defaultdict(list)
    for r in rows(pattern):
        if r.get("Counter_Name") == counter and short(r["Kernel_Name"]) == kernel:
            vals[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    return [sum(v) for v in vals.values()]


# the dominant kernel (most device time): k_chain on the v4 engine, k_level on v3
tot = {k: sum(v) for k, v in per.items() if k in ("k_chain", "k_level", "k_port_stream")}
dom = max(tot, key=tot.get) if tot else "k_level"
wl = bid = None
for f in glob.glob(os.path.join(d, "bench_fetch.json")):
    for ln in open(f):
        if ln.startswith("{"):
            j = json.loads(ln)
            wl, bid = j["config"]["workload"], j.get("build_id")
out = {"kernel": dom, "workload": wl, "build_id": bid,
       "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KB units x1024", "per_kernel": {}}
for k in [dom] + [x for x in ("k_chain", "k_level") if x != dom]:
    fe = pmc("fetch_counter_collection.csv", "FETCH_SIZE", k)
    wr = pmc("write_counter_collection.csv", "WRITE_SIZE", k)
    if not (fe and wr):
        continue
    # counters are in KB (rocprofv3 derived FETCH_SIZE / WRITE_SIZE)
    fb = 2 * 1024 * sum(fe) / len(fe)
    wb = 1024 * sum(wr) / len(wr)
    avg_us = sum(per[k]) / len(per[k]) / 1e3 if per.get(k) else None
    st = per.get(k, [])[-STEADY:]
    out["per_kernel"][k] = {"launches_fetch": len(fe), "launches_write": len(wr),
                            "fetch_bytes_per_launch_corrected": fb, "write_bytes_per_launch": wb,
                            "traffic_bytes_per_launch": fb + wb, "kernel_trace_avg_us": avg_us,
                            "kernel_trace_steady_avg_us": sum(st) / len(st) / 1e3 if st else None}
    print("\nPMC per %s launch: fetch %.1f MB (corrected), write %.1f MB, total %.1f MB" % (k, fb / 1e6, wb / 1e6, (fb + wb) / 1e6))
if dom in out["per_kernel"]:
    out.update(out["per_kernel"][dom])
    with open(os.path.join(d, "pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)
