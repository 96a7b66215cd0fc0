"""Timing of engine path 3 (basic queues with a moving average, serial.hip) on
BASELINE configs[1]'s 32x32 uniform batch: device time, packet-hops/s and a
run-to-run determinism check.  Usage: python tools/ma_timing.py [ppt] [type] [window]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402


def main():
    ppt = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    ma = int(sys.argv[2]) if len(sys.argv) > 2 else gnoc.MOVING_AVG_ARITHMETIC_MEAN
    w = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    tr = gnoc.synthetic_trace(32, 32, 0.005, ppt, seed=1)
    cfg = gnoc.EngineConfig(num_tiles=1024, queue_type=gnoc.QUEUE_BASIC, moving_avg_type=ma, moving_avg_window=w)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    runs = []
    for _ in range(3):
        t0 = time.perf_counter()
        eng.run()
        runs.append((eng.summary()["last_run_ms"], (time.perf_counter() - t0) * 1e3))
        print(f"run: device {runs[-1][0]:.1f} ms, wall {runs[-1][1]:.1f} ms", flush=True)
    a = eng.results()
    eng.run()
    b = eng.results()
    s = a.summary
    ms = min(r[0] for r in runs)
    out = {"workload": f"32x32 uniform load=0.005 pkts/tile={ppt}, basic queue, moving average type {ma} window {w}",
           "packets": len(tr), "mesh_hops": s["mesh_hops"], "levels": s["levels"], "engine_path": s["engine_path"],
           "device_ms": ms, "hops_per_s": s["mesh_hops"] / (ms / 1e3),
           "deterministic": bool(np.array_equal(a.final_ps, b.final_ps) and np.array_equal(a.port_sum_delay,
                                                                                        b.port_sum_delay)),
           "mean_contention_ps": float(a.contention_ps.mean())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
