"""The chain engine's task queues (chain.hip deq_init / deq_next): one queue per XCD
(default), whose hand-offs stay in that XCD's L2, or one shared queue per phase
(GNOC_CH_XCD=0), whose spills and state granules are written through.  Turns are
plain stores in both modes (read by the next launch).  Both must be bit-exact
against the oracle, and against each other on a batch with many spills (short
forced windows) under both hand-off protocols."""
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.test_gpu_lookback import run, same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("lookback", ["0", "1"])
@pytest.mark.parametrize("wps", [5000, 0])
def test_shared_queue_matches_oracle(lookback, wps, monkeypatch):
    monkeypatch.setenv("GNOC_CH_XCD", "0")
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", lookback)
    if wps:
        monkeypatch.setenv("GNOC_WINDOW_PS", str(wps))
    cfg = gnoc.EngineConfig(num_tiles=256)
    tr = gnoc.synthetic_trace(16, 16, 0.03, 300, seed=23)
    got = run(cfg, tr, runs=3)
    same(got, oracle.run(cfg, tr))
    assert got.summary["engine_path"] == 4


@pytest.mark.parametrize("lookback", ["0", "1"])
def test_shared_and_xcd_queues_agree(lookback, monkeypatch):
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", lookback)
    monkeypatch.setenv("GNOC_WINDOW_PS", "20000")
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.01, 400, seed=5)
    monkeypatch.setenv("GNOC_CH_XCD", "0")
    shared = run(cfg, tr)
    monkeypatch.setenv("GNOC_CH_XCD", "1")
    xcd = run(cfg, tr)
    same(xcd, shared)
    assert shared.summary["engine_path"] == 4 and xcd.summary["engine_path"] == 4
