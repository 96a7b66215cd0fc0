"""A 1024-tile proxy of an application trace (configs[3] of BASELINE.json is a
Graphite app capture, which needs Pin; this approximates its traffic shape).

Shared-memory traffic of the pr_l1_pr_l2_dram_directory_msi protocol, as
ShmemMsg::getModeledLength gives it (shmem_msg.cc:100-125): requests / invalidations /
acks carry msg_type + address = 72 bits (2 flits of 64), data replies add a
64-byte cache block = 584 bits (10 flits).  Open loop, seeded:
* every tile issues requests (Bernoulli per cycle) to the home tile of an
  address (uniformly interleaved homes);
* the home answers after a fixed directory delay with a data reply (SH_REP /
  EX_REP, 80 %) or an UPGRADE_REP (72 b), timed from the request's zero-load
  latency;
* a small fraction of requests make the home invalidate with a broadcast
  (ACKwise beyond its sharer pointers), answered by INV_REPs from a few tiles.
Reply times are derived from zero-load latencies, not from the engine: the
trace is a fixed input, like a captured one.

Run from the repo root (oracle, ~10 s):  python tests/golden/make_proxy.py
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
OUT = os.path.join(HERE, "proxy_hashes.json")
REQ_BITS, DATA_BITS = 72, 584
RESULT_FIELDS = ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1",
                 "port_flit", "port_last")


def proxy_trace(W=32, H=32, reqs_per_tile=200, rate=0.004, bcast_frac=0.001, acks=4, dir_delay=10, seed=5):
    rng = np.random.default_rng(seed)
    N = W * H
    # request cycles per tile: geometric gaps of a Bernoulli(rate) process
    gaps = rng.geometric(rate, size=(N, reqs_per_tile)).astype(np.int64)
    t_req = np.cumsum(gaps, axis=1).reshape(-1)
    src = np.repeat(np.arange(N, dtype=np.int64), reqs_per_tile)
    home = rng.integers(0, N, size=src.size)

    def zl(a, b, flits):   # zero-load cycles: (hops + 1)(R + Lk) + F, R = Lk = 1
        return (np.abs(a % W - b % W) + np.abs(a // W - b // W) + 1) * 2 + flits

    data = rng.random(src.size) < 0.8
    rep_bits = np.where(data, DATA_BITS, REQ_BITS)
    t_rep = t_req + zl(src, home, 2) + dir_delay
    pk_t = [t_req, t_rep]
    pk_s = [src, home]
    pk_d = [home, src]
    pk_b = [np.full(src.size, REQ_BITS), rep_bits]
    pk_f = [np.zeros(src.size, np.int64), np.zeros(src.size, np.int64)]
    # invalidation broadcasts from the home, then acks from a few sharers
    inv = np.nonzero(rng.random(src.size) < bcast_frac)[0]
    t_inv = t_req[inv] + zl(src[inv], home[inv], 2) + dir_delay // 2
    pk_t.append(t_inv)
    pk_s.append(home[inv])
    pk_d.append(home[inv])   # ignored for a broadcast
    pk_b.append(np.full(inv.size, REQ_BITS))
    pk_f.append(np.full(inv.size, 2))   # GNOC_PKT_BROADCAST
    sharers = rng.integers(0, N, size=(inv.size, acks))
    for k in range(acks):
        s = sharers[:, k]
        pk_t.append(t_inv + (W + H) * 2 + 2 + k)   # after the tree reaches every tile
        pk_s.append(s)
        pk_d.append(home[inv])
        pk_b.append(np.full(inv.size, REQ_BITS))
        pk_f.append(np.zeros(inv.size, np.int64))
    t = np.concatenate(pk_t)
    order = np.argsort(t, kind="stable")
    return gnoc.Trace((t[order] * 1000).astype(np.uint64), np.concatenate(pk_s)[order].astype(np.uint32),
                      np.concatenate(pk_d)[order].astype(np.uint32), np.concatenate(pk_b)[order].astype(np.uint32),
                      np.concatenate(pk_f)[order].astype(np.uint32))


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).astype(a.dtype.newbyteorder("<"), copy=False).tobytes()).hexdigest()


def trace_hash(tr) -> str:
    h = hashlib.sha256()
    for a in (tr.inject_ps, tr.src, tr.dst, tr.bits, tr.flags):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    from oracle import oracle
    tr = proxy_trace()
    cfg = gnoc.EngineConfig(num_tiles=1024)
    t0 = time.time()
    r = oracle.run(cfg, tr)
    dt = time.time() - t0
    out = {"packets": len(tr), "broadcasts": int((tr.flags & 2).astype(bool).sum()),
           "flits": {"72b": int((tr.bits == REQ_BITS).sum()), "584b": int((tr.bits == DATA_BITS).sum())},
           "trace_sha256": trace_hash(tr), "mg1_uses": int(r.port_mg1.sum()), "oracle_s": round(dt, 1),
           "results": {f: {"sha256": sha(getattr(r, f)),
                           "sum": int(getattr(r, f).astype(np.uint64).sum(dtype=np.uint64))} for f in RESULT_FIELDS}}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(f"proxy trace: {len(tr)} packets, {out['broadcasts']} broadcasts, oracle {dt:.1f} s")


if __name__ == "__main__":
    main()
