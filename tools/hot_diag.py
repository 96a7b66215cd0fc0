"""Why a batch leaves the chain engine: runs a configs[1] batch (uniform or hotspot)
a few times with GNOC_CHAIN_DEBUG=1 (the engine prints the decline flags) and
prints each run's summary.  Usage: python tools/hot_diag.py [hotspot|uniform] [W] [ppt]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GNOC_CHAIN_DEBUG"] = "1"
from graphite_amd import gnoc  # noqa: E402

mix = sys.argv[1] if len(sys.argv) > 1 else "hotspot"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 32
ppt = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
tr = gnoc.synthetic_trace(W, W, 0.005, ppt, seed=1, hotspot_fraction=0.2 if mix == "hotspot" else 0.0, num_hotspots=16)
e = gnoc.Engine(gnoc.EngineConfig(num_tiles=W * W))
e.submit(tr)
for k in range(4):
    e.run()
    s = e.summary()
    print(k, {x: s[x] for x in ("engine_path", "retries", "fallbacks", "windows", "windows_y", "window_ps_x", "window_ps_y",
                                "last_run_ms", "mg1_uses")}, flush=True)
