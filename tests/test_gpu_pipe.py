"""The port pipelines (engine path 6, graphite_amd/csrc/pipe.hip) against the CPU
oracle and against the chain engine (path 4).

One wave per chain port, records handed port to port through LDS rings inside a
segment workgroup and through epoch-tagged HBM records between segments; a
service wave per segment stages the inserts.  Every case asserts the path that
ran, so a silent fallback to the chain engine fails the test.  Integer / ps
arithmetic: exact equality on every output array.
"""
import numpy as np
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.test_gpu_parity import assert_same
from tests.traces import random_trace

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _pipe_on(monkeypatch):
    monkeypatch.setenv("GNOC_PIPE", "1")


def _run(cfg, tr, runs=1):
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    out = []
    for _ in range(runs):
        eng.run()
        out.append((eng.results(), eng.summary()))
    eng.close()
    return out


def _pipe_exact(cfg, tr, runs=1):
    got = _run(cfg, tr, runs)
    ref = oracle.run(cfg, tr)
    mg = int(ref.port_mg1.sum())
    for res, s in got:
        # the pipelines serve batches without the no-gap M/G/1 branch (a bursty batch's
        # first run may merge injection exception tails first: one retry); the branch
        # sends a batch to the chains (test_pipe_declines_mg1_burst_to_chains)
        if mg == 0:
            assert s["engine_path"] == 6 and s["retries"] <= 1 and s["fallbacks"] == 0, s
        assert_same(res, ref)
    return got


@pytest.mark.parametrize("load,ppt", [(0.005, 400), (0.02, 300), (0.05, 300)])
def test_pipe_synthetic_8x8(load, ppt):
    cfg = gnoc.EngineConfig(num_tiles=64)
    _pipe_exact(cfg, gnoc.synthetic_trace(8, 8, load, ppt, seed=11))


@pytest.mark.parametrize("W,H", [(4, 4), (2, 4), (4, 2), (3, 3), (1, 5), (5, 1), (6, 6), (12, 5)])
def test_pipe_mesh_shapes(W, H):
    cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H)
    _pipe_exact(cfg, random_trace(4000, W, H, seed=W * 10 + H, max_cycle=40 * 4000 // (W * H)))


def test_pipe_picosecond_offsets():
    """Inject times off the cycle grid: rho = 1000 tc - t travels with each record."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    _pipe_exact(cfg, random_trace(6000, 8, 8, seed=5, max_cycle=5000, ps_jitter=True))


def test_pipe_ties_at_one_cycle():
    """Many packets arriving in the same cycle: the (time, id) tie order decides."""
    cfg = gnoc.EngineConfig(num_tiles=16)
    tr = random_trace(3000, 4, 4, seed=9, max_cycle=400)
    _pipe_exact(cfg, tr)


@pytest.mark.parametrize("fw,R,tw,lk", [(16, 0, 1.0, 1), (32, 2, 1.0, 1), (128, 1, 150.0, 2), (64, 3, 350.0, 4)])
def test_pipe_flits_and_delays(fw, R, tw, lk):
    cfg = gnoc.EngineConfig(num_tiles=36, flit_width=fw, router_delay=R, tile_width_mm=tw, link_delay=lk)
    tr = random_trace(4000, 6, 6, seed=fw + R, max_cycle=6000, bits_choices=[64, 200, 576, 1500])
    _pipe_exact(cfg, tr)


def test_pipe_self_and_unmodeled():
    cfg = gnoc.EngineConfig(num_tiles=36)
    _pipe_exact(cfg, random_trace(5000, 6, 6, seed=8, max_cycle=5000, self_frac=0.1, unmodeled_frac=0.1))


@pytest.mark.parametrize("S", ["1", "2", "3", "5", "8"])
def test_pipe_segment_sizes(S, monkeypatch):
    """Ports per segment workgroup: S = 1 hands every record through HBM links,
    S = 8 mostly through LDS rings; all exact."""
    monkeypatch.setenv("GNOC_PIPE_S", S)
    cfg = gnoc.EngineConfig(num_tiles=256)
    _pipe_exact(cfg, gnoc.synthetic_trace(16, 16, 0.01, 150, seed=4))


def test_pipe_repeatable_and_resubmit():
    """Runs of one batch give the same bytes (a new link epoch per run); a new
    batch on the same engine is exact too (its links never read the old batch's
    records)."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    a = gnoc.synthetic_trace(8, 8, 0.03, 300, seed=1)
    b = gnoc.synthetic_trace(8, 8, 0.03, 300, seed=2)
    eng = gnoc.Engine(cfg)
    for tr in (a, b, a):
        eng.submit(tr)
        ref = oracle.run(cfg, tr)
        for _ in range(2):
            eng.run()
            s = eng.summary()
            assert s["engine_path"] == 6, s
            assert_same(eng.results(), ref)
    eng.close()


def test_pipe_declines_mg1_burst_to_chains():
    """A cycle-0 burst: the no-gap M/G/1 branch fires in chain ports.  The
    pipelines decline, the chain engine reruns the batch exactly, and later
    runs of the batch go to the chains directly."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(8000, 8, 8, seed=21, max_cycle=600, burst0=300)
    got = _run(cfg, tr, runs=2)
    ref = oracle.run(cfg, tr)
    assert ref.port_mg1.sum() > 0
    (r1, s1), (r2, s2) = got
    assert s1["engine_path"] != 6 and s1["retries"] >= 1, s1
    assert s2["engine_path"] == s1["engine_path"] and s2["retries"] == 0, s2
    assert_same(r1, ref)
    assert_same(r2, ref)


def test_pipe_not_used_off_1ghz():
    """The pipelines serve 1 GHz batches (cycle = 1000 ps); others take the chains."""
    cfg = gnoc.EngineConfig(num_tiles=64, frequency_ghz=0.9)
    tr = random_trace(3000, 8, 8, seed=2, max_cycle=2000, frequency_ghz=0.9)
    (res, s), = _run(cfg, tr)
    assert s["engine_path"] == 4, s
    assert_same(res, oracle.run(cfg, tr))


@pytest.mark.parametrize("hot", [0.0, 0.2])
def test_pipe_matches_chain_engine_32x32(hot, monkeypatch):
    """configs[1]'s mesh and load at 1,000 packets per tile: the pipelines and the
    chain engine give identical bytes."""
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.005, 1000, seed=1, hotspot_fraction=hot, num_hotspots=16)
    (rp, sp), = _run(cfg, tr)
    monkeypatch.setenv("GNOC_PIPE", "0")
    (rc, sc), = _run(cfg, tr)
    assert sp["engine_path"] == 6 and sc["engine_path"] == 4, (sp, sc)
    assert_same(rp, rc)
    assert sp["mesh_hops"] == sc["mesh_hops"]
