"""Fused X+Y chain launch (k_chain_xy) vs the two-launch path and the oracle:
parity on small meshes, then timing on configs[1] (uniform + hotspot).
Usage: python tools/xy_check.py [quick]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402

KEYS = ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last")


def run(W, load, ppt, hot=0.0, runs=10, seed=3, env=None):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        cfg = gnoc.EngineConfig(num_tiles=W * W)
        tr = gnoc.synthetic_trace(W, W, load, ppt, seed=seed, hotspot_fraction=hot, num_hotspots=16)
        e = gnoc.Engine(cfg)
        e.submit(tr)
        info = []
        for _ in range(runs):
            e.run()
            s = e.summary()
            info.append((s["engine_path"], s["chain_protocol"], round(s["last_run_ms"], 3), s["retries"], s["fallbacks"]))
        r = e.results()
        e.close()
        return r, info, tr, cfg
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
    from oracle import oracle
    for W, load, ppt, hot in ((8, 0.05, 300, 0.0), (8, 0.2, 200, 0.0), (16, 0.02, 500, 0.2), (6, 0.05, 300, 0.0)):
        r, info, tr, cfg = run(W, load, ppt, hot)
        ref = oracle.run(cfg, tr)
        bad = [k for k in KEYS[:5] if not np.array_equal(getattr(r, k), getattr(ref, k))]
        print(f"{W}x{W} load {load} hot {hot}: oracle diff {bad} runs {info}", flush=True)
    for W, load, ppt, hot in ((32, 0.005, 1000 if quick else 10000, 0.0), (32, 0.005, 1000 if quick else 10000, 0.2)):
        a, ia, _, _ = run(W, load, ppt, hot, runs=8)
        b, ib, _, _ = run(W, load, ppt, hot, runs=8, env={"GNOC_XY": "0"})
        bad = [k for k in KEYS if not np.array_equal(getattr(a, k), getattr(b, k))]
        print(f"{W}x{W} hot {hot}: fused vs two launches diff {bad}\n  fused {ia}\n  two   {ib}", flush=True)


if __name__ == "__main__":
    main()
