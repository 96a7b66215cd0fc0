"""Oracle pin of BASELINE.json configs[4] at its benched length: the 256-point
design-space sweep (flit width x router delay x tile width -> link delay x offered
load), every point an 8x8 mesh at 2,000 packets per tile
(128,000 packets) with bench.py's seeds (sweep_bench: seed 1 + 7919 i).  The
saturated points (load 0.02 with narrow flits or long delays) drive the history
tree's analytical branch and long queues, the regime the 12-packet GPU test does
not reach.  Each point's eight result arrays are stored as one SHA-256 over their
little-endian bytes (plus the M/G/1 count and the mesh hops, for diagnosis).

Run from the repo root (a few minutes of CPU on 8 cores):
    python tests/golden/make_sweep.py
"""
import hashlib
import itertools
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from graphite_amd import gnoc  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "sweep_hashes.json")
PPT = 2000
SEED = 1
FIELDS = ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit",
          "port_last")


def points():
    """bench.py sweep_points(): (SweepPoint, offered load) for the 256 points."""
    out = []
    for fw, r, tw, load in itertools.product((16, 32, 64, 128), (0, 1, 2, 3), (1.0, 150.0, 250.0, 350.0),
                                             (0.005, 0.01, 0.015, 0.02)):
        out.append((gnoc.SweepPoint(fw, r, int(-(-tw // 100)), tw), load))
    return out


def trace(i, load):
    return gnoc.synthetic_trace(8, 8, load, PPT, seed=SEED + 7919 * i)


def point_hash(res) -> str:
    h = hashlib.sha256()
    for f in FIELDS:
        a = np.ascontiguousarray(getattr(res, f))
        h.update(a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes())
    return h.hexdigest()


def trace_hash(tr) -> str:
    h = hashlib.sha256()
    for a in (tr.inject_ps, tr.src, tr.dst, tr.bits, tr.flags):
        a = np.ascontiguousarray(a)
        h.update(a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes())
    return h.hexdigest()


def _one(i):
    from oracle import oracle
    q, load = points()[i]
    tr = trace(i, load)
    res = oracle.run(q.config(gnoc.EngineConfig(num_tiles=64)), tr)
    return i, point_hash(res), int(res.port_mg1.sum()), int(res.port_count.sum()), trace_hash(tr)


def main():
    t0 = time.time()
    with Pool(8) as pool:
        rows = sorted(pool.map(_one, range(len(points()))))
    out = {"ppt": PPT, "seed": SEED, "fields": list(FIELDS),
           "points": [{"hash": h, "mg1_uses": m, "port_requests": c, "trace_sha256": t} for _, h, m, c, t in rows]}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=0)
    print(f"{len(rows)} points, {sum(r[2] for r in rows)} M/G/1 uses, {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
