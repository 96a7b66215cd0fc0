"""Host side of the design-space sweep (gnoc_create_sweep), on CPU: the block
layout G(p, t) of include/gnoc.h and the (inject_ps, point, id) merge."""
import numpy as np

from graphite_amd import gnoc
from tests.traces import random_trace


def test_global_tiles_are_disjoint_blocks():
    W, H, npts = 4, 3, 7
    bx = int(np.ceil(np.sqrt(npts)))
    seen = set()
    for p in range(npts):
        g = gnoc.sweep_global_tile(p, np.arange(W * H), W, H, bx)
        gx, gy = g % (bx * W), g // (bx * W)
        # the point's tiles form one W x H block, in the point's own row-major order
        assert np.array_equal(gx - gx.min(), np.arange(W * H) % W)
        assert np.array_equal(gy - gy.min(), np.arange(W * H) // W)
        assert gx.min() % W == 0 and gy.min() % H == 0
        seen |= set(g.tolist())
    assert len(seen) == W * H * npts


def test_merge_is_ordered_and_stable_per_point():
    W = H = 4
    trs = [random_trace(500, W, H, seed=s, max_cycle=100) for s in range(5)]
    merged, (pt, lid) = gnoc.sweep_merge(trs, W, H, 3)
    assert np.all(np.diff(merged.inject_ps.astype(np.int64)) >= 0)
    for p, t in enumerate(trs):
        m = pt == p
        assert np.array_equal(lid[m], np.arange(len(t)))          # each point keeps its id order
        assert np.array_equal(merged.inject_ps[m], t.inject_ps)
        g = gnoc.sweep_global_tile(p, t.src, W, H, 3)
        assert np.array_equal(merged.src[m], g)
