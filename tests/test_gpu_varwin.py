"""Variable chain windows (engine.hip adapt_chain_variable): each run of a batch
shape re-cuts every chain's window boundaries from the fills the previous run
measured (up to 8 adaptations), so consecutive runs use different task tables.
Every run must stay bit-exact against the oracle, equal to uniform windows per
chain (GNOC_CH_VARWIN=0), under both hand-off protocols, on uniform and hotspot
traffic (whose bursty central ports make the boundaries most uneven)."""
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.test_gpu_lookback import same

pytestmark = pytest.mark.gpu


def runs(cfg, tr, n):
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    out = []
    for _ in range(n):
        eng.run()
        out.append((eng.results(), eng.summary()))
    eng.close()
    return out


@pytest.mark.parametrize("lookback", ["0", "1"])
@pytest.mark.parametrize("hot", [0.0, 0.2])
def test_every_adaptation_run_matches_oracle(lookback, hot, monkeypatch):
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", lookback)
    cfg = gnoc.EngineConfig(num_tiles=256)
    # (hot ejection ports below saturation: the chains take the batch)
    tr = gnoc.synthetic_trace(16, 16, 0.01, 800, seed=31, hotspot_fraction=hot, num_hotspots=8)
    ref = oracle.run(cfg, tr)
    var = runs(cfg, tr, 10)
    for res, s in var:
        same(res, ref)
        assert s["engine_path"] == 4
    monkeypatch.setenv("GNOC_CH_VARWIN", "0")
    uni = runs(cfg, tr, 3)
    for res, s in uni:
        same(res, ref)
        assert s["engine_path"] == 4
