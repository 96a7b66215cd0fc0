#!/usr/bin/env python3
"""Offline analysis of a chain-stamps dump (tools/chain_stamps.py with CH_STAMPS_DUMP=prefix):
per-chain finish times, the phase's tail, and where the waits sit (window / port).

    python tools/stamps_offline.py gpurun_out/r6b_st_x.npz
"""
import sys

import numpy as np


def main():
    d = np.load(sys.argv[1])
    t, rt, info, tasks, D = d["t"].astype(np.int64), d["rt"].astype(np.int64), d["info"], d["tasks"], d["D"]
    nt, ln, _ = t.shape
    ch, win = (tasks >> 16).astype(np.int64), (tasks & 0xFFFF).astype(np.int64)
    nch = ch.max() + 1
    nW = np.bincount(ch, minlength=nch)
    n = (info & 0xFFFF).astype(np.int64)
    good = (rt[:, 0] > 0) & (rt[:, -1] > 0)
    t0 = rt[good, 0].min()
    # the step end marks (s_memrealtime, 100 MHz): task start ~ first step's end
    end = (rt[:, -1] - t0) / 100.0
    start = (rt[:, 0] - t0) / 100.0
    span = end[good].max()
    print(f"tasks {nt} chains {nch} ports {ln} span {span:.1f} us")
    fin = np.array([end[(ch == c) & good].max() for c in range(nch)])
    work = np.array([n[ch == c].sum() for c in range(nch)])
    order = np.argsort(fin)
    print("chains finishing last (chain, windows, records, finish us):")
    for c in order[-8:]:
        print(f"   {c:3d} nW {nW[c]:4d} recs {work[c]:9d} D {D[c]:10d}  finish {fin[c]:7.1f}")
    print("chains finishing first:")
    for c in order[:4]:
        print(f"   {c:3d} nW {nW[c]:4d} recs {work[c]:9d} D {D[c]:10d}  finish {fin[c]:7.1f}")
    # waits (stamp 3 -> 4) by window decile and by port
    wt = t[:, :, 4] - t[:, :, 3]
    ok = (t[:, :, 4] > 0) & (t[:, :, 3] > 0)
    frac = win / np.maximum(nW[ch] - 1, 1)
    for lo in np.linspace(0, 0.9, 10):
        m = (frac >= lo) & (frac < lo + 0.1 + (1e-9 if lo > 0.85 else 0))
        print(f"  windows {lo:.1f}-{lo + 0.1:.1f}: mean wait/step {wt[m][ok[m]].mean():7.0f} cyc, tasks {m.sum()}")
    pw = [wt[:, i][ok[:, i]].mean() for i in range(ln)]
    print("  wait by port:", " ".join(f"{x:.0f}" for x in pw))
    # the tail: tasks still running in the last 25% of the span, by chain
    tail = good & (end > 0.75 * span)
    cc = np.bincount(ch[tail], minlength=nch)
    print(f"  tasks running in the last quarter: {tail.sum()}; by chain (top): " +
          ", ".join(f"{c}:{cc[c]}" for c in np.argsort(cc)[-10:][::-1]))
    # per-task duration vs when it started
    dur = end - start
    for lo in np.linspace(0, 0.9, 10):
        m = good & (start >= lo * span) & (start < (lo + 0.1) * span)
        if m.sum():
            print(f"  tasks starting at {lo:.1f}-{lo + .1:.1f} of span: {m.sum():5d}, mean duration {dur[m].mean():6.1f} us")


if __name__ == "__main__":
    main()
