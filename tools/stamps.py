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
load = float(sys.argv[3]) if len(sys.argv) > 3 else 0.005
tr = gnoc.synthetic_trace(mesh, mesh, load, ppt, seed=1)
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
d = (st[:, 9] >> 32) & 0xFF
lev = st[:, 9] >> 40
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
    out.append(f"[merge={int(np.median(s[:, 4] - s[:, 12]))}]")
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

# per-level timeline (s_memrealtime: 100 MHz)
rows = []
for L in np.unique(lev):
    m = lev == L
    t0, t1 = st[m, 1].min(), st[m, 11].max()
    span = (t1 - t0) * 10
    busy = ((st[m, 11] - st[m, 1]) * 10).sum()
    rows.append((int(L), int(m.sum()), span / 1000, busy / 1000 / max(span, 1) * 1000))
rows = np.array(rows)
print("levels", len(rows), "sum of spans (us)", round(rows[:, 2].sum(), 1), "mean busy WGs", round(rows[:, 3].mean(), 1))
gaps = []
order = np.argsort([r[0] for r in rows])
ends = {int(L): st[lev == L, 11].max() for L in np.unique(lev)}
starts = {int(L): st[lev == L, 1].min() for L in np.unique(lev)}
ks = sorted(ends)
gap = [(starts[b] - ends[a]) * 10 / 1000 for a, b in zip(ks[:-1], ks[1:])]
print("inter-level gap (us): med", round(float(np.median(gap)), 2), "sum", round(float(np.sum(gap)), 1))
for r in rows[::8]:
    print("  level %2d chunks %5d span %7.1f us  mean busy WGs %6.1f" % tuple(r))
