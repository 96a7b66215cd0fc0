"""Quick GPU check of the port pipelines (engine path 6): small batches against the
oracle, then configs[1] against the chain engine (path 4), with timings.

    python tools/pipe_check.py [--big 0|1] [--S n]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.traces import random_trace  # noqa: E402


def same(a, b):
    bad = []
    for name in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit",
                 "port_last"):
        x, y = getattr(a, name), getattr(b, name)
        if not np.array_equal(x, y):
            d = np.nonzero(x != y)[0]
            bad.append(f"{name}: {d.size} differ, first {d[0]}: {x[d[0]]} vs {y[d[0]]}")
    return bad


def run(cfg, tr, runs=1, env=None):
    old = {}
    for k, v in (env or {}).items():
        old[k] = os.environ.get(k)
        os.environ[k] = v
    try:
        eng = gnoc.Engine(cfg)
        eng.submit(tr)
        ms = []
        for _ in range(runs):
            eng.run()
            ms.append(eng.summary()["last_run_ms"])
        r = eng.results()
        s = eng.summary()
        eng.close()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return r, s, ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", type=int, default=1)
    ap.add_argument("--S", type=str, default="")
    a = ap.parse_args()
    if a.S:
        os.environ["GNOC_PIPE_S"] = a.S
    os.environ.setdefault("GNOC_CHAIN_DEBUG", "1")
    os.environ.setdefault("GNOC_PIPE", "1")
    cases = [
        ("8x8 l0.02", gnoc.EngineConfig(num_tiles=64), gnoc.synthetic_trace(8, 8, 0.02, 300, seed=11)),
        ("8x8 l0.05", gnoc.EngineConfig(num_tiles=64), gnoc.synthetic_trace(8, 8, 0.05, 300, seed=11)),
        ("8x8 jitter", gnoc.EngineConfig(num_tiles=64), random_trace(5000, 8, 8, seed=5, max_cycle=3000, ps_jitter=True)),
        ("6x6 bits", gnoc.EngineConfig(num_tiles=36), random_trace(4000, 6, 6, seed=6, max_cycle=2000,
                                                                   bits_choices=[64, 576, 1024])),
        ("4x4 self", gnoc.EngineConfig(num_tiles=16), random_trace(3000, 4, 4, seed=7, max_cycle=2000, self_frac=0.1)),
        ("16x16 l0.02", gnoc.EngineConfig(num_tiles=256), gnoc.synthetic_trace(16, 16, 0.02, 200, seed=3)),
    ]
    ok = True
    for name, cfg, tr in cases:
        t0 = time.time()
        got, s, _ = run(cfg, tr)
        ref = oracle.run(cfg, tr)
        bad = same(got, ref)
        ok &= not bad
        print(f"{name}: path {s['engine_path']} retries {s['retries']} fallbacks {s['fallbacks']} "
              f"{'OK' if not bad else 'BAD ' + '; '.join(bad)} ({time.time() - t0:.1f} s)", flush=True)
    if a.big:
        cfg = gnoc.EngineConfig(num_tiles=1024)
        for hot in (0.0, 0.2):
            tr = gnoc.synthetic_trace(32, 32, 0.005, 10000, seed=1, hotspot_fraction=hot, num_hotspots=16)
            rp, sp, mp = run(cfg, tr, runs=6)
            rc, sc, mc = run(cfg, tr, runs=6, env={"GNOC_PIPE": "0"})
            bad = same(rp, rc)
            ok &= not bad
            print(f"32x32 hot {hot}: pipe path {sp['engine_path']} ms {[round(x, 3) for x in mp]} | chain path "
                  f"{sc['engine_path']} ms {[round(x, 3) for x in mc]} | {'SAME' if not bad else 'DIFF ' + '; '.join(bad)}",
                  flush=True)
    print("ALL OK" if ok else "FAILURES", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
