"""Broadcast-batch timing: a synthetic 32x32 batch with a
fraction of its packets turned into broadcasts, timed on the GPU; reports the
pass count, device ms and packet-hops/s (a broadcast = N router visits)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from graphite_amd import gnoc  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    ppt = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    fracs = [float(x) for x in sys.argv[3:]] or [0.0, 1e-4, 1e-3]
    base = gnoc.synthetic_trace(W, W, 0.005, ppt, seed=1)
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    rng = np.random.default_rng(7)
    for fr in fracs:
        tr = gnoc.Trace(base.inject_ps, base.src, base.dst, base.bits, base.flags.copy())
        tr.flags[rng.random(len(tr)) < fr] |= gnoc.PKT_BROADCAST
        print(f"-- bcast_frac={fr}: first run", flush=True)
        eng = gnoc.Engine(cfg)
        eng.submit(tr)
        eng.run()
        t0 = time.perf_counter()
        eng.run()
        wall = time.perf_counter() - t0
        s = eng.summary()
        nb, passes = eng.broadcast_info()
        print(f"W={W} bcast_frac={fr} nb={nb} passes={passes} path={s['engine_path']} device_ms={s['last_run_ms']:.2f} "
              f"wall_ms={wall * 1e3:.2f} hops={s['mesh_hops']} Ghops/s={s['mesh_hops'] / wall / 1e9:.3f}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
