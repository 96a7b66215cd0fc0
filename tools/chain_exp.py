#!/usr/bin/env python3
"""k_chain device time of a configs[1] batch with GNOC_CHAIN_EXPERIMENT=1 (the run
stops after the chain phases; results invalid): for timing variants such as the
-DCH_NOWAIT build.  Usage: GNOC_LIB=... python tools/chain_exp.py [mix]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GNOC_CHAIN_EXPERIMENT"] = "1"
from graphite_amd import gnoc  # noqa: E402

mix = sys.argv[1] if len(sys.argv) > 1 else "uniform"
tr = gnoc.synthetic_trace(32, 32, 0.005, 10000, seed=1, hotspot_fraction=0.2 if mix == "hotspot" else 0.0,
                          num_hotspots=16)
eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
eng.submit(tr)
for _ in range(5):
    eng.run()
eng.set_profiling(True)
ms = []
for _ in range(5):
    eng.run()
    ms.append(eng.kernel_stats().get("k_chain", (0, 0))[0])
s = eng.summary()
print(os.path.basename(os.environ.get("GNOC_LIB", "libgnoc.so")), mix, "k_chain ms", [round(x, 3) for x in ms],
      "windows", s["windows"], s["windows_y"], "run ms", round(s["last_run_ms"], 3))
