"""Per-rank device time of a sharded mesh, all ranks in one process on one GPU
(gnoc.LocalShardSet).  Each rank's kernels are timed with HIP events on its own
stream; the ranks run one after another, so each figure is what that rank's GPU
would spend (the all-to-all itself is not included).  Also each rank's k_chain
rate (X / Y hop records per second) against the same mesh on one engine, and
prep_ms = device time minus levels, finalize, chains and window bounds.  Dev
tool, not a test.
usage: python tools/shard_timing.py MESH NRANKS [PPT] [LOAD]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from graphite_amd import gnoc  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ppt = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
load = float(sys.argv[4]) if len(sys.argv) > 4 else (0.002 if W == 64 else 0.005)
cfg = gnoc.EngineConfig(num_tiles=W * W)
tr = gnoc.synthetic_trace(W, W, load, ppt, seed=1)


def chain_rate(eng_stats, res):
    """X / Y hop records per second of k_chain (LEFT, RIGHT, DOWN, UP port requests)."""
    pc = res.port_count.reshape(-1, 6)
    recs = int(pc[:, 1:5].sum())
    ms = eng_stats["k_chain"][0]
    return recs, ms, (recs / (ms * 1e-3) if ms else 0.0)


# the same mesh on one engine: the per-rank k_chain rates are compared with this one
one = gnoc.Engine(cfg)
one.submit(tr)
for _ in range(3):
    one.run()
one.set_profiling(True)
one.run()
one_recs, one_ms, one_rate = chain_rate(one.kernel_stats(), one.results())
one.close()
ss = gnoc.LocalShardSet(cfg, n)
ss.submit(tr)
ss.run()
ss.set_profiling(True)
ss.run()
rows = []
for r, e in enumerate(ss.engs):
    ks = e.kernel_stats()
    tot = sum(v[0] for v in ks.values())
    res = e.results()
    pc = res.port_count.reshape(-1, 6)
    recs, cms, rate = chain_rate(ks, res)
    rows.append({"rank": r, "device_ms": round(tot, 3), "k_level_ms": round(ks["k_level"][0], 3),
                 "k_chain_ms": round(cms, 3), "k_chain_recs_per_s": rate,
                 "k_chain_rate_vs_one_gpu": round(rate / one_rate, 3) if one_rate else None,
                 "prep_ms": round(tot - ks["k_level"][0] - ks["k_finalize"][0] - cms - ks["k_win_bounds"][0], 3),
                 "mesh_hops": int(pc[:, :5].sum()), "send_MB": round(sum(ss.su[r]) * 16 / 1e6, 1),
                 "kernels": {k: round(v[0], 3) for k, v in ks.items() if v[1]}})
hops = ss.engs[0].summary()["mesh_hops"]
worst = max(x["device_ms"] for x in rows)
print(json.dumps({"mesh": W, "ranks": n, "packets": len(tr), "mesh_hops": hops, "max_rank_device_ms": worst,
                  "one_gpu_k_chain_ms": round(one_ms, 3), "one_gpu_k_chain_recs_per_s": one_rate,
                  "projected_hops_per_s_excl_exchange": hops / (worst * 1e-3), "per_rank": rows}))
ss.close()
