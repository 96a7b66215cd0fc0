"""Per-run chain-engine window sizes (per phase), retries and device time of the
configs[1] batch run repeatedly (the engine resizes its windows from each run's
measured fill).  Dev tool.  usage: python tools/window_trace.py [runs] [ppt]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
from graphite_amd import gnoc  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ppt = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
tr = gnoc.synthetic_trace(32, 32, 0.005, ppt, seed=1)
eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
eng.submit(tr)
for k in range(runs):
    eng.run()
    s = eng.summary()
    print(k, f"{s['last_run_ms']:.3f} ms", "windows", s["windows"], s["windows_y"], "D", s["window_ps_x"], s["window_ps_y"],
          "retries", s["retries"], "fallbacks", s["fallbacks"], "path", s["engine_path"], flush=True)
