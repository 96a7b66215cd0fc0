#!/usr/bin/env python3
"""Per-step phase timing of the chain engine (rows kernel, chain.hip CH_STAMP 0-7).

Needs a -DCH_STAMPS build (tools/build_variant.sh stamps -DCH_STAMPS, then
GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so).  Runs one configs[1]-style
batch (settled windows), reads k_chain's per-(task, port) s_memtime stamps and
prints where a step's time goes:
  rows  = [0 -> 1] state prefetch issue + the merged stream's rows from LDS
  bscan = [1 -> 2] per-row max-plus scans and route-field totals
  land  = [2 -> 3] the next port's inserts into LDS
  wait  = [3 -> 4] polling the predecessor window's state of this port
  slow  = [4 -> 5] early publish, spill-ins (slow path)
  emit  = [5 -> 6] recurrence, kept records, turn / spill stores
  post  = [6 -> 7] late publish, port counters, prefetches of later ports
  gap   = [7 -> next 0]
Usage: python tools/chain_stamps.py [W] [load] [ppt] [mix]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GNOC_STAMPS"] = "1"

import numpy as np  # noqa: E402

from graphite_amd import gnoc  # noqa: E402

NAMES = ("rows", "bscan", "land", "wait", "slow", "emit", "post")


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    load = float(sys.argv[2]) if len(sys.argv) > 2 else 0.005
    ppt = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    hot = 0.2 if (len(sys.argv) > 4 and sys.argv[4] == "hotspot") else 0.0
    tr = gnoc.synthetic_trace(W, W, load, ppt, seed=1, hotspot_fraction=hot, num_hotspots=16)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=W * W))
    eng.submit(tr)
    for _ in range(4):
        eng.run()
    eng.set_profiling(True)
    eng.run()
    s = eng.summary()
    print("summary", s)
    print("kernel_ms", {k: round(v[0], 3) for k, v in eng.kernel_stats().items() if v[0] > 0})
    fn = eng.lib.gnoc_debug_chain_stamps
    fn.restype = ctypes.c_int
    for phase in (0, 1):
        cnt = ctypes.c_size_t(0)
        geom = (ctypes.c_uint32 * 4)()
        fn(eng._h, phase, None, 0, ctypes.byref(cnt), geom)
        _, nt, ln, _ = list(geom)
        buf = np.zeros(cnt.value, np.uint64)
        fn(eng._h, phase, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cnt.value, ctypes.byref(cnt), geom)
        st = buf.reshape(nt, ln, 16)
        t = st[:, :, :8].astype(np.int64)
        info = st[:, :, 8]
        n = (info & 0xFFFF).astype(np.int64)
        itot = ((info >> 16) & 0xFFFF).astype(np.int64)
        nkeep = ((info >> 32) & 0xFFFF).astype(np.int64)
        slow = (info >> 63).astype(bool)
        ok = (t[:, :-1, 7] > 0) & (t[:, :-1, 0] > 0) & (t[:, 1:, 0] > 0) & (t[:, :-1, 5] > 0)
        d = {NAMES[k]: t[:, :-1, k + 1] - t[:, :-1, k] for k in range(7)}
        d["gap"] = t[:, 1:, 0] - t[:, :-1, 7]
        print(f"phase {'XY'[phase]}: tasks {nt} len {ln} steps {ok.sum()}")
        tot = np.zeros(ok.sum())
        for k, v in d.items():
            x = v[ok]
            tot += x
            print(f"  {k:6s} mean {x.mean():8.0f}  med {np.median(x):8.0f}  p90 {np.percentile(x, 90):8.0f}  cyc")
        print(f"  step   mean {tot.mean():8.0f}  med {np.median(tot):8.0f}")
        nn = n[:, :-1][ok]
        print(f"  records/step mean {nn.mean():.0f} p50 {np.median(nn):.0f} p90 {np.percentile(nn, 90):.0f} max {n.max()}"
              f"  inserts/step mean {itot[:, :-1][ok].mean():.1f}  kept/step mean {nkeep[:, :-1][ok].mean():.0f}"
              f"  slow-path steps {slow[:, :-1][ok].mean() * 100:.1f}%")
        rows = (nn + 63) // 64
        for r in range(1, 13):
            m = rows == r
            if m.sum() > 100:
                print(f"    {r:2d} rows: {m.sum():7d} steps, mean step {tot[m].mean():7.0f}  emit {d['emit'][ok][m].mean():6.0f}"
                      f"  bscan {d['bscan'][ok][m].mean():6.0f}  rows {d['rows'][ok][m].mean():6.0f}")
        good = (t[:, 0, 0] > 0) & (t[:, -1, 7] > 0)
        task_t = t[:, -1, 7] - t[:, 0, 0]
        print(f"  task duration med {np.median(task_t[good]):.0f} cyc")
        # occupancy over the phase from s_memrealtime (100 MHz, shared by the XCDs; the
        # s_memtime counters are per XCD): running tasks per 1/50 of the phase
        rt = st[:, :, 9].astype(np.int64)
        good &= (rt[:, 0] > 0) & (rt[:, -1] > 0)
        t0, t1 = rt[good][:, 0].min(), rt[good][:, -1].max()
        print(f"  span of phase {(t1 - t0) / 100:.1f} us (s_memrealtime, step end marks)")
        st_, en_ = rt[good][:, 0] - t0, rt[good][:, -1] - t0
        task_t = en_ - st_
        nb = 50
        edges = np.linspace(0, t1 - t0, nb + 1)
        run = np.array([((st_ < edges[b + 1]) & (en_ > edges[b])).sum() for b in range(nb)])
        busy = task_t[good].sum() / (run.max() * (t1 - t0))
        print(f"  running tasks per 1/{nb} of the phase: " + " ".join(str(x) for x in run))
        print(f"  task-slot utilisation (task time / (peak running x span)): {busy:.3f}")
        if os.environ.get("CH_STAMPS_DUMP"):
            # raw per-step stamps for offline analysis: s_memtime stamps 0-7 (low 32 bits),
            # the step's s_memrealtime end mark, the record counts, and the task table
            tn = ctypes.c_size_t(0)
            tf = eng.lib.gnoc_debug_chain_tasks
            tf.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t,
                           ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
            tf(eng._h, phase, None, 0, ctypes.byref(tn), None, 0)
            tab = np.zeros(tn.value, np.uint32)
            dl = np.zeros(4096, np.uint64)
            tf(eng._h, phase, tab.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), tn.value, ctypes.byref(tn),
               dl.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), dl.size)
            np.savez_compressed(f"{os.environ['CH_STAMPS_DUMP']}_{'xy'[phase]}.npz", t=st[:, :, :8].astype(np.uint32),
                                rt=st[:, :, 9], info=st[:, :, 8], tasks=tab, D=dl)


if __name__ == "__main__":
    main()
