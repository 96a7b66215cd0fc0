"""One batch on the port pipelines with GNOC_PIPE_DEBUG (wave states printed on give-up)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ppt = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
hot = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
runs = int(sys.argv[4]) if len(sys.argv) > 4 else 1
os.environ.setdefault("GNOC_PIPE_DEBUG", "31")
os.environ.setdefault("GNOC_CHAIN_DEBUG", "1")
os.environ.setdefault("GNOC_PIPE", "1")
tr = gnoc.synthetic_trace(W, W, 0.005, ppt, seed=1, hotspot_fraction=hot, num_hotspots=16)
eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=W * W))
eng.submit(tr)
for r in range(runs):
    t0 = time.time()
    eng.run()
    s = eng.summary()
    print(f"run {r}: path {s['engine_path']} ms {s['last_run_ms']:.3f} retries {s['retries']} fallbacks {s['fallbacks']} "
          f"wall {time.time() - t0:.2f} s", flush=True)
