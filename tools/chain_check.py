#!/usr/bin/env python3
"""GPU-box check of the v4 chain engine against the CPU oracle on a set of
traces, with forced window sizes (GNOC_WINDOW_SHIFT) that put many window
edges (spills) into every chain.  Prints one line per case; exits non-zero on
the first mismatch."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from graphite_amd import gnoc  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.traces import random_trace  # noqa: E402


def check(name, cfg, tr, shift=None):
    if shift:
        os.environ["GNOC_WINDOW_SHIFT"] = str(shift)
    else:
        os.environ.pop("GNOC_WINDOW_SHIFT", None)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    t0 = time.perf_counter()
    try:
        eng.run()
    except gnoc.GnocError as ex:
        print(f"{name:40s} shift={shift} ERROR {ex}", flush=True)
        eng.close()
        return False
    dt = time.perf_counter() - t0
    got = eng.results()
    s = eng.summary()
    eng.close()
    ref = oracle.run(cfg, tr)
    bad = []
    for f in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit",
              "port_last"):
        a, b = getattr(got, f), getattr(ref, f)
        if not np.array_equal(a, b):
            i = np.nonzero(a != b)[0]
            bad.append(f"{f}: {i.size} differ, first {i[0]} gpu {a[i[0]]} ref {b[i[0]]}")
    print(f"{name:40s} shift={shift} path={s['engine_path']} pkts={len(tr)} hops={s['mesh_hops']} "
          f"gpu_ms={s['last_run_ms']:.2f} wall={dt*1e3:.1f} W={s['windows']}/{s['window_shift']} "
          f"retry={s['retries']} fb={s['fallbacks']} {'OK' if not bad else 'FAIL'}", flush=True)
    for b in bad:
        print("   ", b, flush=True)
    return not bad


def main():
    ok = True
    c64 = gnoc.EngineConfig(num_tiles=64)
    for sh in (None, 14, 17, 20):
        ok &= check("8x8 synthetic 0.02", c64, gnoc.synthetic_trace(8, 8, 0.02, 300, seed=11), sh)
        ok &= check("8x8 synthetic 0.05", c64, gnoc.synthetic_trace(8, 8, 0.05, 300, seed=11), sh)
    ok &= check("8x8 random burst (M/G/1)", c64, random_trace(20000, 8, 8, seed=3, max_cycle=300, burst0=400))
    ok &= check("8x8 random self/unmodeled", c64,
                random_trace(6000, 8, 8, seed=5, max_cycle=3000, self_frac=0.1, unmodeled_frac=0.1), 16)
    ok &= check("6x6 flits mix", gnoc.EngineConfig(num_tiles=36),
                random_trace(8000, 6, 6, seed=7, max_cycle=20000, bits_choices=[72, 576, 584, 1088]), 17)
    ok &= check("4x4 jitter", gnoc.EngineConfig(num_tiles=16),
                random_trace(3000, 4, 4, seed=9, max_cycle=20000, ps_jitter=True), 15)
    ok &= check("1x5", gnoc.EngineConfig(mesh_width=1, mesh_height=5, num_tiles=5),
                random_trace(2000, 1, 5, seed=2, max_cycle=20000), 16)
    ok &= check("5x1", gnoc.EngineConfig(mesh_width=5, mesh_height=1, num_tiles=5),
                random_trace(2000, 5, 1, seed=2, max_cycle=20000), 16)
    ok &= check("3x7", gnoc.EngineConfig(mesh_width=3, mesh_height=7, num_tiles=21),
                random_trace(6000, 3, 7, seed=4, max_cycle=20000), 16)
    c1 = gnoc.EngineConfig(num_tiles=1024)
    for sh in (None, 18):
        ok &= check("32x32 uniform 0.005 ppt=300", c1, gnoc.synthetic_trace(32, 32, 0.005, 300, seed=1), sh)
    ok &= check("32x32 hotspot 0.005 ppt=300", c1,
                gnoc.synthetic_trace(32, 32, 0.005, 300, seed=1, hotspot_fraction=0.2, num_hotspots=16))
    ok &= check("32x32 uniform 0.01 ppt=200", c1, gnoc.synthetic_trace(32, 32, 0.01, 200, seed=2), 19)
    print("ALL OK" if ok else "FAILURES", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
