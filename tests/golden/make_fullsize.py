"""Full-size oracle pins of the BASELINE.json headline configurations.

configs[1]: 32x32 emesh_hop_by_hop, uniform and hotspot traffic, offered load
0.005, 10,000 packets per tile (10.24 M packets); configs[2]: 64x64, load
0.002, 10,000 packets per tile (40.96 M packets) -- the traces bench.py times.
The expected outputs are the CPU oracle's (oracle/gnoc_oracle.c, pinned by the
reference's history_tree KAT and differential tests, tests/test_oracle.py).
Far too large to commit, so each result array is stored as a SHA-256 of its
little-endian bytes plus its sum ("a seed plus a SHA-256
of the results").  The trace itself is regenerated from its seed on the GPU
box and checked against the stored trace hash first.

Run from the repo root (about 8 minutes of CPU):
    python tests/golden/make_fullsize.py            # all cases
    python tests/golden/make_fullsize.py 32x32      # cases whose name starts so
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from graphite_amd import gnoc  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "fullsize_hashes.json")

# name -> (W, H, offered load, packets per tile, seed, hotspot fraction): bench.py's workloads
CASES = {
    "32x32_uniform_l0.005_ppt10000": (32, 32, 0.005, 10000, 1, 0.0),
    "32x32_hotspot_l0.005_ppt10000": (32, 32, 0.005, 10000, 1, 0.2),
    "64x64_uniform_l0.002_ppt10000": (64, 64, 0.002, 10000, 1, 0.0),
    # configs[1]'s uniform batch behind a cycle-0 burst of 4 packets per tile (uniform
    # random destinations, seed 7): the history tree's analytical branch
    # (queue_model_history_tree.cc:58-64) serves requests in injection AND mesh ports
    "32x32_burst4_l0.005_ppt10000": (32, 32, 0.005, 10000, 1, 0.0, 4),
}
BURST_SEED = 7
RESULT_FIELDS = ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1",
                 "port_flit", "port_last")


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<"), copy=False).tobytes()).hexdigest()


def trace_of(name):
    W, H, load, ppt, seed, hot = CASES[name][:6]
    tr = gnoc.synthetic_trace(W, H, load, ppt, seed=seed, hotspot_fraction=hot, num_hotspots=16)
    burst = CASES[name][6] if len(CASES[name]) > 6 else 0
    if not burst:
        return tr
    rng = np.random.default_rng(BURST_SEED)
    N = W * H
    bs = np.repeat(np.arange(N, dtype=np.uint32), burst)
    bd = rng.integers(0, N, bs.size).astype(np.uint32)
    cat = lambda a, b: np.concatenate([a.astype(b.dtype), b])
    fl = tr.flags if tr.flags is not None else np.zeros(len(tr), np.uint32)
    return gnoc.Trace(cat(np.zeros(bs.size, np.uint64), tr.inject_ps), cat(bs, tr.src), cat(bd, tr.dst),
                      cat(np.full(bs.size, 576, np.uint32), tr.bits), cat(np.zeros(bs.size, np.uint32), fl))


def trace_hash(tr) -> str:
    h = hashlib.sha256()
    for a in (tr.inject_ps, tr.src, tr.dst, tr.bits):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def digest(res) -> dict:
    return {f: {"sha256": sha(getattr(res, f)), "sum": int(getattr(res, f).astype(np.uint64).sum(dtype=np.uint64))}
            for f in RESULT_FIELDS}


def main(only=None):
    from oracle import oracle
    out = {}
    if os.path.exists(OUT):
        with open(OUT) as fh:
            out = json.load(fh)
    for name, spec in CASES.items():
        W, H, load, ppt, seed, hot = spec[:6]
        if only and not name.startswith(only):
            continue
        tr = trace_of(name)
        cfg = gnoc.EngineConfig(num_tiles=W * H)
        t0 = time.time()
        r = oracle.run(cfg, tr)
        dt = time.time() - t0
        hops = int(r.port_count.reshape(-1, 6)[:, :5].sum())
        out[name] = {"W": W, "H": H, "load": load, "ppt": ppt, "seed": seed, "hotspot_fraction": hot,
                     "num_hotspots": 16, "burst_per_tile": spec[6] if len(spec) > 6 else 0, "packets": len(tr), "mesh_hops": hops, "trace_sha256": trace_hash(tr),
                     "mg1_uses": int(r.port_mg1.sum()), "results": digest(r), "oracle_s": round(dt, 1)}
        print(f"{name}: {len(tr)} packets, {hops} mesh hops, oracle {dt:.1f} s", flush=True)
        with open(OUT, "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
