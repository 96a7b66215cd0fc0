import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from graphite_amd import gnoc
W = H = 4
cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H, flit_width=64)
n0 = 1024
t = np.concatenate([np.arange(n0, dtype=np.uint64), np.full(3, n0 + 1, np.uint64)]) * np.uint64(1000)
dst = (np.arange(t.size, dtype=np.uint32) % (W * H - 1)) + 1
tr = gnoc.Trace(t, np.zeros(t.size, np.uint32), dst, np.full(t.size, 64, np.uint32), np.zeros(t.size, np.uint32))
eng = gnoc.Engine(cfg)
eng.submit(tr)
for r in range(3):
    eng.run()
    s = eng.summary()
    print("run", r, {k: s[k] for k in ("engine_path", "retries", "fallbacks", "windows", "windows_y", "window_ps_x", "window_ps_y", "chain_protocol")}, flush=True)
