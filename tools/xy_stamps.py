#!/usr/bin/env python3
"""Fused X+Y chain launch: where the time goes (a -DCH_STAMPS build:
tools/build_variant.sh stamps -DCH_STAMPS; GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so).
Per 1/50 of the launch: running X tasks, running Y tasks, Y tasks waiting for the X
tasks they depend on; task durations; the Y tasks' wait at their start.
Usage: python tools/xy_stamps.py [lag] [mix]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GNOC_STAMPS"] = "1"
if len(sys.argv) > 1:
    os.environ["GNOC_XY_LAG"] = sys.argv[1]

import numpy as np  # noqa: E402

from graphite_amd import gnoc  # noqa: E402


def main():
    hot = 0.2 if (len(sys.argv) > 2 and sys.argv[2] == "hotspot") else 0.0
    tr = gnoc.synthetic_trace(32, 32, 0.005, 10000, seed=1, hotspot_fraction=hot, num_hotspots=16)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
    eng.submit(tr)
    for _ in range(12):
        eng.run()
        if eng.summary()["chain_protocol"] & 0x200 and _ >= 6:
            break
    eng.run()
    s = eng.summary()
    print("summary", {k: s[k] for k in ("engine_path", "chain_protocol", "last_run_ms", "windows", "windows_y")})
    fn = eng.lib.gnoc_debug_chain_stamps
    cnt = ctypes.c_size_t(0)
    geom = (ctypes.c_uint32 * 4)()
    fn(eng._h, 2, None, 0, ctypes.byref(cnt), geom)
    _, nt, ln, nx = list(geom)
    buf = np.zeros(cnt.value, np.uint64)
    fn(eng._h, 2, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cnt.value, ctypes.byref(cnt), geom)
    tab = np.zeros(nt, np.uint32)
    c2 = ctypes.c_size_t(0)
    eng.lib.gnoc_debug_xy_tasks(eng._h, tab.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), nt, ctypes.byref(c2))
    st = buf.reshape(nt, ln, 16).astype(np.int64)
    isy = (tab >> 31).astype(bool)
    t0r = st[:, 0, 10]                 # task start (after dequeue), s_memrealtime
    wend = np.where(isy, st[:, 0, 11], t0r)
    tend = st[:, -1, 9]                # last step's end mark
    good = (t0r > 0) & (tend > 0) & (wend > 0)
    base = t0r[good].min()
    T = tend[good].max() - base
    print(f"tasks {nt} (X {nx}, Y {nt - nx}), all stamped {good.sum()}; launch span {T / 100:.1f} us")
    a, w, e = t0r - base, wend - base, tend - base
    nb = 50
    edges = np.linspace(0, T, nb + 1)
    for name, m in (("X run", ~isy & good), ("Y wait", isy & good), ("Y run", isy & good)):
        lo = a if name != "Y run" else w
        hi = e if name != "Y wait" else w
        row = [int(((lo[m] < edges[b + 1]) & (hi[m] > edges[b])).sum()) for b in range(nb)]
        print(f"  {name:7s}: " + " ".join(str(x) for x in row))
    yw = (w - a)[isy & good] / 100.0
    print(f"  Y wait at start: mean {yw.mean():.1f} us, p50 {np.median(yw):.1f}, p90 {np.percentile(yw, 90):.1f}, "
          f"max {yw.max():.1f}")
    for name, m, lo in (("X", ~isy & good, a), ("Y", isy & good, w)):
        d = (e - lo)[m] / 100.0
        print(f"  {name} task run: mean {d.mean():.1f} us p50 {np.median(d):.1f} p90 {np.percentile(d, 90):.1f}")
    xe = e[~isy & good]
    print(f"  X tasks: last end at {xe.max() / T:.3f} of the span; Y tasks: first start {w[isy & good].min() / T:.3f}")


if __name__ == "__main__":
    main()
