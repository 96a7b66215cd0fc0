"""The chain engine's look-back hand-off protocol (GNOC_CHAIN_LOOKBACK=1, chain.hip
task_lb): a window composes the nearest inclusive state of its port with the
aggregates of the windows after it.  Bit-exact against the oracle, and equal to
the serial protocol, on batches chosen to stress it: short forced windows
(many spills across windows, deep look-backs), cycle-0 bursts (the history
tree's "no gap yet" state, where the protocol must wait serially), several mesh
shapes and network frequencies."""
import numpy as np
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.traces import random_trace

pytestmark = pytest.mark.gpu

FIELDS = ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit",
          "port_last")


def run(cfg, tr, runs=2):
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    for _ in range(runs):
        eng.run()
    got = eng.results()
    eng.close()
    return got


def same(got, ref):
    for k in FIELDS:
        a, b = getattr(got, k), getattr(ref, k)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            raise AssertionError(f"{k}: {bad.size} differ, first {bad[0]}: {a[bad[0]]} vs {b[bad[0]]}")


@pytest.mark.parametrize("wps", [3000, 20000, 200000, 2000000])
@pytest.mark.parametrize("load", [0.02, 0.08])
def test_forced_short_windows_match_oracle(wps, load, monkeypatch):
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", "1")
    monkeypatch.setenv("GNOC_WINDOW_PS", str(wps))
    cfg = gnoc.EngineConfig(num_tiles=256)
    tr = gnoc.synthetic_trace(16, 16, load, 200, seed=wps % 97 + int(load * 100))
    got = run(cfg, tr)
    same(got, oracle.run(cfg, tr))
    # the look-back protocol declines exactly where the serial one does (e.g. an M/G/1
    # request before a port's first gap), and otherwise runs on the chain engine
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", "0")
    ser = run(cfg, tr)
    assert got.summary["engine_path"] == ser.summary["engine_path"]
    assert wps == 2000000 or load > 0.05 or got.summary["engine_path"] == 4


@pytest.mark.parametrize("W,H", [(8, 8), (5, 3), (1, 9), (9, 1), (12, 7)])
def test_mesh_shapes_bursts(W, H, monkeypatch):
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", "1")
    monkeypatch.setenv("GNOC_WINDOW_PS", "50000")
    cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H)
    tr = random_trace(6000, W, H, seed=W * 31 + H, max_cycle=3000, burst0=30)
    same(run(cfg, tr), oracle.run(cfg, tr))


@pytest.mark.parametrize("freq", [0.9, 1.5])
def test_non_unit_frequency(freq, monkeypatch):
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", "1")
    cfg = gnoc.EngineConfig(num_tiles=256, frequency_ghz=freq)
    tr = gnoc.synthetic_trace(16, 16, 0.02, 300, seed=int(freq * 10), frequency_ghz=freq)
    got = run(cfg, tr)
    assert got.summary["engine_path"] == 4
    same(got, oracle.run(cfg, tr))


def test_protocols_agree_32x32_hotspot(monkeypatch):
    """Both protocols, several runs each (window adaptation in between), on a
    32x32 hotspot batch: byte-identical results."""
    tr = gnoc.synthetic_trace(32, 32, 0.005, 1500, seed=3, hotspot_fraction=0.2, num_hotspots=16)
    cfg = gnoc.EngineConfig(num_tiles=1024)
    out = {}
    for lb in ("0", "1"):
        monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", lb)
        out[lb] = run(cfg, tr, runs=3)
        assert out[lb].summary["engine_path"] == 4
    same(out["1"], out["0"])
