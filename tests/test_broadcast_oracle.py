"""Oracle restatement of the broadcast tree (emesh_hop_by_hop.cc:163-221,
router_model.cc:70-108): closed-form and counting properties on CPU.

The network layer of the oracle is pinned by citation; these
properties pin what the tree must do independently of the event loop:
every tile receives once, zero-load = (H+1)(R+Lk) + F, each router charges
the max over its ports to every port, and a port's request count is the
number of broadcasts whose tree uses it."""
import numpy as np

from graphite_amd import gnoc
from oracle import oracle
from tests.traces import random_trace


def tree_ports(W, H, s):
    """(tile, port) requests of one broadcast from s, restated from the reference branch."""
    sx, sy = s % W, s // W
    out = []
    for t in range(W * H):
        cx, cy = t % W, t // W
        if cy >= sy and cy + 1 < H:
            out.append((t, gnoc.PORT_UP))
        if cy <= sy and cy >= 1:
            out.append((t, gnoc.PORT_DOWN))
        if cy == sy:
            if cx >= sx and cx + 1 < W:
                out.append((t, gnoc.PORT_RIGHT))
            if cx <= sx and cx >= 1:
                out.append((t, gnoc.PORT_LEFT))
        out.append((t, gnoc.PORT_SELF))
    return out


def one_broadcast(W, H, s, t0=0, bits=576, **kw):
    return gnoc.Trace(np.array([t0], np.uint64), np.array([s], np.uint32), np.array([0], np.uint32),
                      np.array([bits], np.uint32), np.array([gnoc.PKT_BROADCAST], np.uint32))


def test_single_broadcast_zero_load():
    for W, H, s in [(4, 3, 5), (1, 5, 2), (5, 1, 0), (3, 3, 8), (6, 4, 13)]:
        cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H)
        r = oracle.run(cfg, one_broadcast(W, H, s, t0=7000))
        sx, sy = s % W, s // W
        hops = np.array([abs(t % W - sx) + abs(t // W - sy) for t in range(W * H)])
        zl = (hops + 1) * 2000 + 9000
        assert np.array_equal(r.bcast_zero_load_ps[0], zl)
        assert np.array_equal(r.bcast_final_ps[0], 7000 + zl)
        far = int(np.argmax(zl))
        assert r.final_ps[0] == 7000 + zl[far] and r.contention_ps[0] == 0
        # 2N records: 1 injection + 2N - 1 router requests
        pc = r.port_count.reshape(-1, 6)
        assert pc[:, :5].sum() == 2 * W * H - 1 and pc[:, 5].sum() == 1
        want = np.zeros_like(pc)
        for t, p in tree_ports(W, H, s):
            want[t, p] += 1
        want[s, gnoc.PORT_INJ] = 1
        assert np.array_equal(pc, want)


def test_back_to_back_broadcasts_serialise_once():
    """Two broadcasts from one tile at one time: the second waits F cycles at
    injection and then follows the first F cycles behind at every port."""
    W, H = 4, 4
    cfg = gnoc.EngineConfig(num_tiles=16)
    tr = gnoc.Trace(np.zeros(2, np.uint64), np.array([6, 6], np.uint32), np.zeros(2, np.uint32),
                    np.full(2, 576, np.uint32), np.full(2, gnoc.PKT_BROADCAST, np.uint32))
    r = oracle.run(cfg, tr)
    assert np.array_equal(r.bcast_final_ps[1], r.bcast_final_ps[0] + 9000)
    assert np.array_equal(r.bcast_zero_load_ps[1], r.bcast_zero_load_ps[0])


def test_broadcast_only_load_contends():
    """Broadcasts alone build queueing; every receipt's contention is >= 0."""
    W, H = 4, 4
    cfg = gnoc.EngineConfig(num_tiles=16)
    rng = np.random.default_rng(2)
    n = 40
    tr = gnoc.Trace(np.sort(rng.integers(0, 30, n)).astype(np.uint64) * 1000, rng.integers(0, 16, n).astype(np.uint32),
                    np.zeros(n, np.uint32), np.full(n, 576, np.uint32), np.full(n, gnoc.PKT_BROADCAST, np.uint32))
    r = oracle.run(cfg, tr)
    assert r.port_sum_delay.sum() > 0
    # contention of each receipt = final - inject - zero-load, never negative
    assert np.all(r.bcast_final_ps >= tr.inject_ps[:, None] + r.bcast_zero_load_ps)


def test_unmodeled_broadcast_and_contention_off():
    cfg = gnoc.EngineConfig(num_tiles=9)
    tr = random_trace(300, 3, 3, seed=4, max_cycle=100, unmodeled_frac=0.2, bcast_frac=0.3)
    r = oracle.run(cfg, tr)
    bc = (tr.flags & gnoc.PKT_BROADCAST) != 0
    um = (tr.flags & gnoc.PKT_UNMODELED) != 0
    rows = np.nonzero(bc)[0]
    for k, i in enumerate(rows):
        if um[i]:
            assert np.all(r.bcast_final_ps[k] == tr.inject_ps[i]) and np.all(r.bcast_zero_load_ps[k] == 0)
    off = oracle.run(gnoc.EngineConfig(num_tiles=9, contention_enabled=False), tr)
    assert np.array_equal(off.bcast_final_ps, tr.inject_ps[rows][:, None] + off.bcast_zero_load_ps)


def test_expand_broadcasts_is_netsend():
    tr = random_trace(50, 3, 3, seed=9, bcast_frac=0.2)
    ex = gnoc.expand_broadcasts(tr, 9)
    nb = int(((tr.flags & gnoc.PKT_BROADCAST) != 0).sum())
    assert len(ex) == len(tr) + 8 * nb
    assert not np.any(ex.flags & gnoc.PKT_BROADCAST)
    assert np.all(np.diff(ex.inject_ps.astype(np.int64)) >= 0)
