"""Diagnostic: per-phase s_memtime stamps of the v3 level kernel (GNOC_STAMPS=1).
Prints median cycles per phase by port direction. Dev tool, not a test."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GNOC_STAMPS"] = "1"
from graphite_amd import gnoc  # noqa: E402

mesh = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ppt = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
tr = gnoc.synthetic_trace(mesh, mesh, 0.005, ppt, seed=1)
eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=mesh * mesh))
eng.submit(tr)
eng.run()
lib = eng.lib
lib.gnoc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
n = ctypes.c_size_t()
lib.gnoc_debug_stamps(eng._h, None, 0, ctypes.byref(n))
buf = np.zeros(n.value * 16, np.uint64)
lib.gnoc_debug_stamps(eng._h, buf.ctypes.data, buf.size, ctypes.byref(n))
st = buf.reshape(-1, 16).astype(np.int64)
st = st[st[:, 8] > 0]
j = st[:, 9] & 0xFFFFFFFF
d = st[:, 9] >> 32
names = ["", "desc", "keys", "search", "load+merge", "scan", "pub+lookback", "process", "tail"]
print("chunks", st.shape[0], "summary", eng.summary(), "records/chunk median", int(np.median(st[:, 10])))
for dirn, label in ((5, "INJ"), (2, "RIGHT"), (1, "LEFT"), (4, "UP"), (3, "DOWN"), (0, "SELF")):
    m = (d == dirn) & (j > 0) & (st[:, 7] > 0)
    if not m.any():
        continue
    s = st[m]
    out = [f"{names[k]}={int(np.median(s[:, k] - s[:, k - 1]))}" for k in range(3, 9)]
    tot = np.median(s[:, 8] - s[:, 0])
    lb = s[:, 13] - s[:, 5]
    spins = s[:, 14] & 0xFFFFFFFF
    dist = s[:, 14] >> 32
    out.append(f"[lookback={int(np.median(lb))} p90={int(np.percentile(lb, 90))} spins med={int(np.median(spins))} "
               f"p90={int(np.percentile(spins, 90))} incl-dist med={int(np.median(dist))} p90={int(np.percentile(dist, 90))}]")
    out.append(f"[load={int(np.median(s[:, 11] - s[:, 3]))} exc={int(np.median(s[:, 12] - s[:, 11]))} "
               f"merge={int(np.median(s[:, 4] - s[:, 12]))}]")
    print(f"{label:6s} n={m.sum():6d} total={int(tot)} " + " ".join(out))

# predecessor timing (s_memrealtime, 100 MHz -> ns x10): take and aggregate publish of chunk g-1 vs g
gi = np.nonzero((j > 0) & (st[:, 15] > 0))[0]
prev = gi - 1
okp = st[prev, 15] > 0
gi, prev = gi[okp], prev[okp]
dt_take = (st[prev, 1] - st[gi, 1]) * 10
dt_pub = (st[prev, 15] - st[gi, 15]) * 10
print("pred take - own take (ns): med", int(np.median(dt_take)), "p10", int(np.percentile(dt_take, 10)), "p90", int(np.percentile(dt_take, 90)), "frac pred later", round(float((dt_take > 0).mean()), 3))
print("pred pub  - own pub  (ns): med", int(np.median(dt_pub)), "p10", int(np.percentile(dt_pub, 10)), "p90", int(np.percentile(dt_pub, 90)), "frac pred later", round(float((dt_pub > 0).mean()), 3))
own = (st[gi, 15] - st[gi, 1]) * 10
print("own take->pub (ns): med", int(np.median(own)), "p90", int(np.percentile(own, 90)))
