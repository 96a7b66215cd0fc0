#!/usr/bin/env python3
"""Per-step phase timing of the chain engine (GNOC_STAMPS=1 build path).

Runs one configs[1]-style batch, reads k_chain's per-(task, port) s_memtime
stamps and prints where a step's time goes:
  scan  = [A] prefetch issue + segment loads + block scan
  wait  = wave 0 polling the predecessor window's state of this port
  d     = rest of [D] up to barrier 2
  emit  = [E] recurrence + stores + reductions (to barrier 3)
  F     = [F] wave 0's late publish and port counters
  gap   = end of [F] -> start of the next step
Usage: python tools/chain_stamps.py [W] [load] [ppt]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GNOC_STAMPS"] = "1"

import numpy as np  # noqa: E402

from graphite_amd import gnoc  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    load = float(sys.argv[2]) if len(sys.argv) > 2 else 0.005
    ppt = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    tr = gnoc.synthetic_trace(W, W, load, ppt, seed=1)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=W * W))
    eng.submit(tr)
    eng.run()
    eng.set_profiling(True)
    eng.run()
    s = eng.summary()
    print("summary", s)
    print("kernel_ms", {k: round(v[0], 3) for k, v in eng.kernel_stats().items() if v[0] > 0})
    lib = eng.lib
    fn = lib.gnoc_debug_chain_stamps
    fn.restype = ctypes.c_int
    for phase in (0, 1):
        cnt = ctypes.c_size_t(0)
        geom = (ctypes.c_uint32 * 4)()
        fn(eng._h, phase, None, 0, ctypes.byref(cnt), geom)
        nch, nW, ln, sh = list(geom)
        buf = np.zeros(cnt.value, np.uint64)
        fn(eng._h, phase, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cnt.value, ctypes.byref(cnt), geom)
        st = buf.reshape(nW * nch, ln, 16).astype(np.int64)
        t = st[:, :, :6]
        info = buf.reshape(nW * nch, ln, 16)[:, :, 6]
        n = (info & 0xFFFF).astype(np.int64)
        itot = ((info >> 16) & 0xFFFF).astype(np.int64)
        spill = (info >> 63).astype(bool)
        ok = (st[:, :-1, 9] > 0) & (t[:, :-1, 0] > 0) & (t[:, 1:, 0] > 0)
        d = {
            "A": st[:, :-1, 7] - st[:, :-1, 0],
            "walk": st[:, :-1, 8] - st[:, :-1, 7],
            "bscan": st[:, :-1, 1] - st[:, :-1, 8],
            "wait": t[:, :-1, 2] - t[:, :-1, 1],
            "d": t[:, :-1, 3] - t[:, :-1, 2],
            "Epre": st[:, :-1, 12] - st[:, :-1, 3],
            "Eloop": st[:, :-1, 13] - st[:, :-1, 12],
            "Epost": st[:, :-1, 4] - st[:, :-1, 13],
            "F": st[:, :-1, 9] - st[:, :-1, 4],
            "gap": t[:, 1:, 0] - st[:, :-1, 9],
        }
        print(f"phase {'XY'[phase]}: chains {nch} windows {nW} len {ln} shift {sh} steps {ok.sum()}")
        tot = np.zeros(ok.sum())
        for k, v in d.items():
            x = v[ok]
            tot += x
            print(f"  {k:6s} mean {x.mean():8.0f}  med {np.median(x):8.0f}  p90 {np.percentile(x, 90):8.0f}  cyc")
        print(f"  step   mean {tot.mean():8.0f}  med {np.median(tot):8.0f}")
        print(f"  records/step mean {n[:, :-1][ok].mean():.0f} max {n.max()}  inserts/step mean {itot[:, :-1][ok].mean():.1f}"
              f"  slow-path steps {spill[:, :-1][ok].mean()*100:.1f}%")
        task_t = st[:, -1, 9] - t[:, 0, 0]
        good = t[:, 0, 0] > 0
        print(f"  task duration med {np.median(task_t[good]):.0f} cyc; span of phase {t[good][:, :, 0].max() - t[good][:, 0, 0].min()} cyc")
        # records per step by window: where the LDS capacity is used
        nw_ = n[:, :-1].reshape(nW, nch, ln - 1)
        mx = nw_.max(axis=(1, 2))
        top = np.argsort(mx)[::-1][:8]
        print("  busiest windows (index: max records/step):", ", ".join(f"{q}: {mx[q]}" for q in top),
              f"| 99th pct of per-window max {np.percentile(mx, 99):.0f}, median {np.median(mx):.0f}")
        # per chain: the fullest step (would per-chain windows help?)
        cm = nw_.max(axis=(0, 2))
        print("  per-chain max records/step: sorted", np.sort(cm).tolist())
        # wait vs window index
        w_idx = np.repeat(np.arange(nW), nch)
        for q in (0, 1, 2, nW // 2, nW - 1):
            m = (w_idx == q)
            if m.any():
                print(f"    window {q:4d}: wait mean {d['wait'][m][ok[m]].mean():8.0f} step mean {tot.mean():8.0f}")


if __name__ == "__main__":
    main()
