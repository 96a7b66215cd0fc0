"""Exception tails of the injection level merged into order before the chains
(chain.hip k_exc_merge): a batch whose injection queues serve cycle-0 bursts by
M/G/1 (the history tree's analytical branch, queue_model_history_tree.cc:58-64)
stays on the chain engine, bit-exact against the oracle.  M/G/1 requests in mesh
ports send the batch to k_chain's MG instantiation (the no-gap prefix served
serially); where that declines too (an M/G/1-served spill) the
Y and SELF levels run on k_level (engine path 5) or the batch on the level
engine (path 1).  Every path is bit-exact."""
import numpy as np
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.traces import random_trace

pytestmark = pytest.mark.gpu

FIELDS = ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit")


def same(got, ref):
    for k in FIELDS:
        a, b = getattr(got, k), getattr(ref, k)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            raise AssertionError(f"{k}: {bad.size} differ, first {bad[0]}: {a[bad[0]]} vs {b[bad[0]]}")


def burst_trace(W, H, per_tile, tail, seed, max_cycle=4000):
    """Every tile injects `per_tile` packets at cycle 0, then a light random tail."""
    rng = np.random.default_rng(seed)
    N = W * H
    src0 = np.repeat(np.arange(N, dtype=np.uint32), per_tile)
    t1 = np.sort(rng.integers(1, max_cycle, tail)).astype(np.uint64) * np.uint64(1000)
    src = np.concatenate([src0, rng.integers(0, N, tail).astype(np.uint32)])
    t = np.concatenate([np.zeros(src0.size, np.uint64), t1])
    dst = rng.integers(0, N, src.size).astype(np.uint32)
    return gnoc.Trace(t, src, dst, np.full(src.size, 576, np.uint32), np.zeros(src.size, np.uint32))


@pytest.mark.parametrize("W,H,per_tile,seed", [(8, 8, 6, 1), (8, 8, 20, 2), (5, 3, 12, 3), (16, 16, 4, 4)])
def test_cycle0_burst_mg1_exact_over_reruns(W, H, per_tile, seed):
    """Cycle-0 bursts from every tile: M/G/1 requests in injection AND mesh ports.
    Bit-exact against the oracle on three runs of the batch, whichever engine path
    each run takes (printed).  The 16 x 16 case pins its path: after the first run
    the batch runs on k_chain's MG instantiation (engine path 4, chain_protocol bit
    10) with no rerun."""
    cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H)
    tr = burst_trace(W, H, per_tile, 4000, seed)
    ref = oracle.run(cfg, tr)
    assert ref.port_mg1.sum() > 0
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    paths = []
    for r in range(3):
        eng.run()
        got = eng.results()
        same(got, ref)
        s = got.summary
        paths.append(s["engine_path"])
        if W == 16 and r:
            assert s["engine_path"] == 4 and s["chain_protocol"] & 0x400, s
            assert s["retries"] == 0 and s["fallbacks"] == 0, s
    eng.close()
    print("engine paths", paths, "mg1 uses", int(ref.port_mg1.sum()))


def star_trace(W, H, ax, ay, seed, tail=3000):
    """Tile (ax, ay) injects 6 packets at cycle 0, one along each of 6 paths (no mesh
    port gets more than 2 of them, so only its injection queue backs up beyond one
    service time: packets 3-6 are served by M/G/1 there); random traffic from cycle 500."""
    rng = np.random.default_rng(seed)
    a = ay * W + ax
    dst0 = [(ax + 2, ay), (ax - 2, ay), (ax, ay + 2), (ax, ay - 2), (ax + 1, ay + 1), (ax - 1, ay - 1)]
    d0 = np.array([y * W + x for x, y in dst0], np.uint32)
    t1 = np.sort(rng.integers(500, 5000, tail)).astype(np.uint64) * np.uint64(1000)
    t = np.concatenate([np.zeros(6, np.uint64), t1])
    src = np.concatenate([np.full(6, a, np.uint32), rng.integers(0, W * H, tail).astype(np.uint32)])
    dst = np.concatenate([d0, rng.integers(0, W * H, tail).astype(np.uint32)])
    return gnoc.Trace(t, src, dst, np.full(t.size, 576, np.uint32), np.zeros(t.size, np.uint32))


@pytest.mark.parametrize("W,ax,ay", [(8, 4, 4), (16, 7, 9), (8, 2, 5)])
def test_injection_only_mg1_runs_on_chain(W, ax, ay):
    """M/G/1 only in one injection queue: the first run's streamed injection level
    declines (the run stops, one retry with the level on k_level), that level's
    exception tails are merged and the run reruns on the chains (a second retry);
    later runs do both up front; bit-exact throughout."""
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    tr = star_trace(W, W, ax, ay, seed=W + ax)
    ref = oracle.run(cfg, tr)
    assert ref.port_mg1.sum() > 0
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    for k in range(3):
        eng.run()
        got = eng.results()
        same(got, ref)
        s = got.summary
        assert s["engine_path"] == 4, s
        assert s["fallbacks"] == 0
        assert s["retries"] == (2 if k == 0 else 0), s
    eng.close()


def test_saturated_mg1_matches_either_path():
    """test_gpu_parity's saturated batch (M/G/1 also in mesh ports): still exact."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(20000, 8, 8, seed=3, max_cycle=300, burst0=400)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    got = eng.results()
    eng.close()
    same(got, oracle.run(cfg, tr))


def column_burst_trace(W, H, ax, ay, k, seed, tail=3000):
    """Tile (ax, ay) injects k packets at cycle 0, all to tiles of its own column (they
    turn UP / DOWN at the source router: the injection queue and the source's Y ports
    back up, its X ports see nothing of the burst); random traffic from cycle 500."""
    rng = np.random.default_rng(seed)
    a = ay * W + ax
    ys = [y for y in range(H) if y != ay]
    d0 = np.array([rng.choice(ys) * W + ax for _ in range(k)], np.uint32)
    t1 = np.sort(rng.integers(500, 5000, tail)).astype(np.uint64) * np.uint64(1000)
    t = np.concatenate([np.zeros(k, np.uint64), t1])
    src = np.concatenate([np.full(k, a, np.uint32), rng.integers(0, W * H, tail).astype(np.uint32)])
    dst = np.concatenate([d0, rng.integers(0, W * H, tail).astype(np.uint32)])
    return gnoc.Trace(t, src, dst, np.full(t.size, 576, np.uint32), np.zeros(t.size, np.uint32))


@pytest.mark.parametrize("W,ax,ay,k", [(8, 3, 4, 14), (8, 6, 1, 20), (16, 9, 8, 24)])
def test_y_only_mg1_keeps_x_on_chain(W, ax, ay, k):
    """M/G/1 in Y ports only: the first run's Y chains decline for the analytical
    branch and the batch reruns on k_chain's MG instantiation (engine path 4, one
    retry, chain_protocol bit 10), or -- when the serial prefix itself declines -- its
    Y and SELF levels run on k_level (engine path 5, one fallback).  Bit-exact either way."""
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    tr = column_burst_trace(W, W, ax, ay, k, seed=W * 7 + k)
    ref = oracle.run(cfg, tr)
    mg = ref.port_mg1.reshape(-1, 6)
    assert mg[:, [3, 4]].sum() > 0                       # M/G/1 in DOWN / UP ports
    assert mg[:, [1, 2]].sum() == 0                      # none in LEFT / RIGHT
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    paths = []
    for r in range(3):
        eng.run()
        got = eng.results()
        same(got, ref)
        s = got.summary
        paths.append(int(s["engine_path"]))
        if s["engine_path"] == 4:
            assert s["fallbacks"] == 0 and s["chain_protocol"] & 0x400, s
            # (first run: the MG rerun, and possibly one for the windows the burst overflowed
            # and one for the streamed injection level, which declines on the burst's
            # source queue)
            assert (1 <= s["retries"] <= 3) if r == 0 else s["retries"] == 0, s
        else:
            assert s["engine_path"] == 5, s
            assert s["fallbacks"] == (1 if r == 0 else 0), s
    eng.close()
    print("engine paths", paths)


def test_overflow_then_y_mg1_decline_is_exact(monkeypatch):
    """a first run whose windows overflow LDS (forced long windows,
    a dense column burst) reruns with halved windows, and that rerun meets the Y
    ports' M/G/1 branch: the run must end exact on the chains (MG instantiation) or
    on the Y levels, never return an internal rerun code."""
    monkeypatch.setenv("GNOC_WINDOW_PS", "4000000")
    W = 8
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    tr = column_burst_trace(W, W, 3, 4, 16, seed=71, tail=20000)
    ref = oracle.run(cfg, tr)
    assert ref.port_mg1.reshape(-1, 6)[:, [3, 4]].sum() > 0
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    s = eng.summary()
    same(eng.results(), ref)
    assert s["retries"] >= 1 and s["engine_path"] in (1, 4, 5), s
    eng.run()
    same(eng.results(), ref)
    eng.close()
    print("summary", s)


def test_refused_exception_slot_with_y_mg1_is_exact():
    """an injection queue whose M/G/1 exception tail (2,600 records into
    one RIGHT slot) is longer than k_exc_merge merges (XM = 2,048), together with
    M/G/1 in Y ports (a column burst).  A decline after the MG instantiation's Y
    chains clears only the SELF slots' exception counts; the refused slot's tail is
    still served in order by the level engine.  Bit-exact on every run."""
    W = 8
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    rng = np.random.default_rng(77)
    big = 4 * W + 1
    t_big = np.zeros(2600, np.uint64)
    col = column_burst_trace(W, W, 3, 2, 20, seed=78, tail=4000)
    t = np.concatenate([t_big, col.inject_ps])
    src = np.concatenate([np.full(2600, big, np.uint32), col.src])
    dst = np.concatenate([np.full(2600, 4 * W + 6, np.uint32), col.dst])
    order = np.argsort(t, kind="stable")
    tr = gnoc.Trace(t[order], src[order], dst[order], np.full(t.size, 576, np.uint32), np.zeros(t.size, np.uint32))
    ref = oracle.run(cfg, tr)
    mg = ref.port_mg1.reshape(-1, 6)
    assert mg[big, 5] > 2048 and mg[:, [3, 4]].sum() > 0
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    paths = []
    for _ in range(3):
        eng.run()
        got = eng.results()
        same(got, ref)
        paths.append(int(got.summary["engine_path"]))
    eng.close()
    print("engine paths", paths)


def test_inj_stream_gap_on_block_boundary():
    """The streamed injection level (chain.hip k_inj_stream) walks a slot in blocks
    of 1,024 records.  Here tile 0's injection queue is busy without a gap for
    exactly one block (one 1-flit packet per cycle from cycle 0), idles for a cycle,
    and the next block opens with a 3-packet burst whose third packet would be
    served by M/G/1 (X > t + p) had the queue never idled.  The idle cycle falls on
    the block boundary, where the block-relative tail is clamped to the block's
    first cycle: the stream must still see the gap (queue_model_history_tree.cc:79-86)
    and not decline (a false decline reruns the batch and keeps it off the stream)."""
    W = H = 4
    cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H, flit_width=64)
    n0 = 1024
    t = np.concatenate([np.arange(n0, dtype=np.uint64), np.full(3, n0 + 1, np.uint64)]) * np.uint64(1000)
    dst = (np.arange(t.size, dtype=np.uint32) % (W * H - 1)) + 1
    src = np.zeros(t.size, np.uint32)
    tr = gnoc.Trace(t, src, dst, np.full(t.size, 64, np.uint32), np.zeros(t.size, np.uint32))
    ref = oracle.run(cfg, tr)
    assert ref.port_mg1.sum() == 0
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    for _ in range(2):
        eng.run()
        got = eng.results()
        same(got, ref)
        s = got.summary
        assert s["engine_path"] == 4 and s["retries"] == 0 and s["fallbacks"] == 0, s
    eng.close()
