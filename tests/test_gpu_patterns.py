"""The reference generator's non-uniform traffic patterns (synthetic_network.cc
:288-341) on the GPU engine vs the oracle, bit-exact.  Fixed-destination
patterns concentrate load on few X / Y chains (transpose, tornado) -- the
non-uniform port loads the chain engine's window sizing and the level engine's
chunk splitter see least under uniform traffic."""
import pytest

from graphite_amd import gnoc
from tests.test_gpu_parity import assert_same, run_both

pytestmark = pytest.mark.gpu

PATTERNS = ["bit_complement", "shuffle", "transpose", "tornado", "nearest_neighbor"]


@pytest.mark.parametrize("pattern", PATTERNS)
def test_pattern_32x32(pattern):
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.002, 200, seed=7, pattern=pattern)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)
    assert got.summary["mesh_hops"] == int(ref.port_count.reshape(-1, 6)[:, :5].sum())


@pytest.mark.parametrize("pattern", PATTERNS)
@pytest.mark.parametrize("load", [0.01, 0.08])
def test_pattern_8x8(pattern, load):
    """Up to saturation (the M/G/1 branch then fires, and the chain engine hands
    the batch to the level engine)."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, load, 300, seed=3, pattern=pattern)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


def test_tornado_32x32_hotspot_mix_forced_windows(monkeypatch):
    """Tornado plus a hotspot fraction, with small forced chain windows (many
    window edges and spills per chain)."""
    monkeypatch.setenv("GNOC_WINDOW_SHIFT", "17")
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.002, 150, seed=9, pattern="tornado", hotspot_fraction=0.1)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


@pytest.mark.parametrize("wps", [98_765, 1_234_567])
def test_odd_window_lengths(monkeypatch, wps):
    """Window lengths that are not powers of two (the engine sizes each phase's
    windows from the fill it measured): records sit on window edges at odd
    offsets; hotspot mix, bit-exact."""
    monkeypatch.setenv("GNOC_WINDOW_PS", str(wps))
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.004, 120, seed=11, hotspot_fraction=0.2)
    got, ref = run_both(cfg, tr)
    assert got.summary["engine_path"] == 4 and got.summary["window_ps_x"] == wps
    assert_same(got, ref)


def test_adapted_windows_repeat_exactly():
    """Runs after the first resize the windows from the measured fill (per phase);
    every run gives the same bytes as the oracle."""
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.005, 300, seed=13)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    sizes, res = [], []
    for _ in range(3):
        eng.run()
        s = eng.summary()
        sizes.append((s["window_ps_x"], s["window_ps_y"]))
        res.append(eng.results())
    eng.close()
    ref = oracle_run(cfg, tr)
    for r in res:
        assert_same(r, ref)
    assert sizes[1] != sizes[0] or sizes[2] == sizes[1]


def oracle_run(cfg, tr):
    from oracle import oracle
    return oracle.run(cfg, tr)


@pytest.mark.parametrize("pch", [1024, 4096, 16384])
def test_prep_chunk_sizes(monkeypatch, pch):
    """The prep workgroups' trace chunk (GNOC_PREP_CHUNK, default 8192) only
    changes how k_classify / k_scatter4 split the trace: same bytes."""
    monkeypatch.setenv("GNOC_PREP_CHUNK", str(pch))
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.004, 60, seed=23, hotspot_fraction=0.1)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)
