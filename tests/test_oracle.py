"""The CPU oracle, pinned before it is trusted.

* the reference's own known-answer test, tests/unit/history_tree/history_tree.cc:9-20
  (committed as tests/golden/history_tree_kat.json);
* differential checks against oracle/_ref, i.e. the reference's real
  IntervalTree (interval_tree.cc), QueueModelMG1 (queue_model_m_g_1.cc) and
  Latency/Time (time_types.h) compiled from /root/reference (skipped where the
  reference tree is absent, e.g. on the GPU box);
* committed network-level golden vectors (tests/golden/*.npz, produced by
  tests/golden/make_golden.py from this oracle once it passed the above).
"""
import json
import os
import random

import numpy as np
import pytest

from oracle import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_history_tree_kat():
    kat = json.load(open(os.path.join(GOLD, "history_tree_kat.json")))
    q = oracle.Queue(100, True, 1)
    for t, p, expect in kat["packets"]:
        assert q.compute(t, p) == expect


def _ref_or_skip():
    r = oracle.ref_lib()
    if r is None:
        pytest.skip("oracle/_ref not built (reference tree absent)")
    return r


def test_ref_kat():
    r = _ref_or_skip()
    kat = json.load(open(os.path.join(GOLD, "history_tree_kat.json")))
    q = r.ref_queue_create(100, 1, 1)
    got = [r.ref_queue_compute(q, t, p) for t, p, _ in kat["packets"]]
    r.ref_queue_destroy(q)
    assert got == [e for *_, e in kat["packets"]]


@pytest.mark.parametrize("seed", range(6))
def test_queue_vs_reference_tree(seed):
    """Sorted-array free list + M/G/1 == real AVL IntervalTree + QueueModelMG1,
    including out-of-order arrivals, the analytical branch and pruning."""
    r = _ref_or_skip()
    L = oracle.lib()
    rng = random.Random(seed)
    for _ in range(400):
        ml = rng.choice([2, 3, 4, 7, 100])
        an = rng.choice([0, 1])
        qo = L.orc_queue_create(ml, an, 1)
        qr = r.ref_queue_create(ml, an, 1)
        t = 0
        for _ in range(rng.randint(1, 250)):
            mode = rng.random()
            if mode < 0.6:
                t += rng.choice([0, 0, 1, 2, 3, 9, 40])
            tt = t if mode < 0.85 else max(0, t - rng.randint(0, 60))
            p = rng.randint(1, 12)
            assert L.orc_queue_compute(qo, tt, p) == r.ref_queue_compute(qr, tt, p)
        assert L.orc_queue_mg1_uses(qo) == r.ref_queue_mg1_uses(qr)
        L.orc_queue_destroy(qo)
        r.ref_queue_destroy(qr)


def test_time_conversions_vs_reference():
    r = _ref_or_skip()
    L = oracle.lib()
    rng = random.Random(1)
    for f in (1.0, 0.9, 1.5, 0.7, 2.0, 0.333, 1.1):
        for _ in range(2000):
            c = rng.choice([rng.randint(0, 100), rng.randint(0, 10**9), rng.randint(0, 2**40)])
            assert L.orc_lat_to_ps(c, f) == r.ref_lat_to_ps(c, f)
            p = rng.choice([rng.randint(0, 10**5), rng.randint(0, 10**12), rng.randint(0, 2**50)])
            assert L.orc_time_to_cycles(p, f) == r.ref_time_to_cycles(p, f)


@pytest.mark.parametrize("name", sorted(f[:-4] for f in os.listdir(GOLD) if f.endswith(".npz")) if os.path.isdir(GOLD) else [])
def test_network_golden(name):
    from graphite_amd.gnoc import EngineConfig, Trace
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    cfg = EngineConfig(**json.loads(str(z["cfg"])))
    tr = Trace(z["inject_ps"], z["src"], z["dst"], z["bits"], z["flags"])
    res = oracle.run(cfg, tr)
    for k in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1"):
        assert np.array_equal(getattr(res, k), z[k]), k


# --- the other queue models of QueueModel::create (queue_model.cc:18-38) -------------

def _sorted_stream(seed, n=3000, burst=40):
    rng = np.random.default_rng(seed)
    t = np.sort(rng.integers(0, n // 3, n))
    t[:burst] = 0
    p = rng.integers(1, 12, n)
    return np.sort(t), p


@pytest.mark.parametrize("L", [2, 3, 4, 7, 100])
@pytest.mark.parametrize("interleaving", [False, True])
def test_history_list_is_the_tree_on_in_order_requests(L, interleaving):
    """In-order requests never fit an earlier gap, so the list (with or without
    interleaving) gives the tree's delays and M/G/1 uses; its after-insert
    pruning makes max_list_size 2 behave like the tree's >= 3."""
    for seed in range(4):
        t, p = _sorted_stream(seed)
        ql = oracle.Queue(L, True, kind=2, interleaving=interleaving)
        qt = oracle.Queue(max(L, 3), True, kind=0)
        dl = [ql.compute(int(a), int(b)) for a, b in zip(t, p)]
        dt = [qt.compute(int(a), int(b)) for a, b in zip(t, p)]
        assert dl == dt
        assert ql.mg1_uses == qt.mg1_uses


def test_basic_is_the_fifo_recurrence():
    for seed in range(4):
        t, p = _sorted_stream(seed)
        qb = oracle.Queue(kind=1)
        X, want = 0, []
        for a, b in zip(t, p):
            want.append(max(X - int(a), 0))
            X = max(X, int(a)) + int(b)
        assert [qb.compute(int(a), int(b)) for a, b in zip(t, p)] == want
        assert qb.mg1_uses == 0


@pytest.mark.parametrize("ma", [1, 2, 3])
@pytest.mark.parametrize("w", [1, 2, 5, 64, 100])
def test_moving_average_matches_reference_source(ma, w):
    """MovingAverage<UInt64>::compute (moving_average.h, arithmetic / geometric /
    median) restated in the oracle == the reference's own header compiled in
    oracle/_ref, number for number, over cycle streams with repeats, steps and gaps."""
    r = oracle.ref_lib()
    if r is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(ma * 1000 + w)
    steps = rng.choice([0, 0, 1, 2, 3, 9, 40, 1000, 123457], size=20000)
    xs = (np.cumsum(steps) + int(rng.integers(1, 50))).tolist()
    q = oracle.Queue(kind=1)
    q.set_moving_avg(ma, w)
    h = r.ref_ma_create(ma, w)
    try:
        got = [q.moving_avg(x) for x in xs]
        want = [int(r.ref_ma_compute(h, x)) for x in xs]
    finally:
        r.ref_ma_destroy(h)
    assert got == want


def test_basic_with_moving_average_queue():
    """QueueModelBasic::computeQueueDelay with a moving average
    (queue_model_basic.cc:35-61): ref = MA(t); d = max(Q - ref, 0);
    Q = max(Q, ref) + p -- against a direct restatement over the reference's MA."""
    r = oracle.ref_lib()
    if r is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for ma, w in ((1, 64), (3, 8), (2, 4)):
        t, p = _sorted_stream(ma + w)
        qb = oracle.Queue(kind=1)
        qb.set_moving_avg(ma, w)
        h = r.ref_ma_create(ma, w)
        Q, want = 0, []
        for a, b in zip(t.tolist(), p.tolist()):
            ref = int(r.ref_ma_compute(h, a))
            want.append(max(Q - ref, 0))
            Q = max(Q, ref) + b
        r.ref_ma_destroy(h)
        assert [qb.compute(int(a), int(b)) for a, b in zip(t, p)] == want


def test_history_list_out_of_order_uses_gaps():
    """Out of order (not produced on this path, but the restatement covers it):
    a request fits an earlier gap, and with interleaving spans gaps."""
    q = oracle.Queue(100, False, kind=2, interleaving=False)
    assert q.compute(10, 5) == 0      # busy [10, 15), gap [0, 10)
    assert q.compute(2, 3) == 0       # fits the gap
    assert q.compute(12, 4) == 3      # waits for 15


@pytest.mark.parametrize("W,load,ppt,seed", [(8, 0.05, 400, 1), (8, 0.3, 250, 2), (6, 0.1, 300, 3)])
def test_network_walk_with_reference_queue_objects(W, load, ppt, seed):
    """The oracle's event loop with every history-tree queue replaced by the
    reference's own IntervalTree + QueueModelMG1 objects (oracle/_ref, compiled from
    its sources; bench.py's CPU baseline runs this) gives the restatement's results
    exactly: per packet and per port, M/G/1 uses included."""
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built (no /root/reference)")
    from graphite_amd import gnoc
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    tr = gnoc.synthetic_trace(W, W, load, ppt, seed=seed)
    a = oracle.run(cfg, tr)
    b = oracle.run(cfg, tr, ref_queues=True)
    for k in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit",
              "port_last"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    if load >= 0.3:
        assert a.port_mg1.sum() > 0
