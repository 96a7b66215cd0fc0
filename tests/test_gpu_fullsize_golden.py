"""BASELINE.json headline configurations at FULL size, bit-exact against the
CPU oracle ("a seed plus a SHA-256 of the results").

tests/golden/fullsize_hashes.json holds, per workload, the SHA-256 of every
output array of the oracle run (final_ps, zero_load_ps, contention_ps and the
per-port sum / count / M/G/1 / flit / last arrays), made in the build
container by tests/golden/make_fullsize.py (the oracle needs 2.5 min for a
32x32 batch and 25 min for the 64x64 one).  Here the trace is regenerated
from its seed (its own SHA-256 checked first), run through the engine, and
every result array must hash identically:
* configs[1]: 32x32 uniform and hotspot, load 0.005, 10,000 packets per tile
  (10.24 M packets, 228 M mesh hops) -- the bench workload;
* configs[1]'s uniform batch behind a cycle-0 burst of 4 packets per tile,
  whose M/G/1 requests (injection and mesh ports) the pin counts;
* configs[2]: 64x64 uniform, load 0.002, 10,000 packets per tile (40.96 M
  packets, 1.79 G mesh hops), on one engine and sharded over 8 row / column
  band ranks (gnoc.LocalShardSet, all ranks on the one test GPU).
"""
import json
import os

import numpy as np
import pytest

from graphite_amd import gnoc
from tests.golden.make_fullsize import RESULT_FIELDS, sha, trace_hash, trace_of

pytestmark = pytest.mark.gpu

with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_hashes.json")) as _fh:
    GOLD = json.load(_fh)


def _check(name, res):
    g = GOLD[name]["results"]
    bad = [f for f in RESULT_FIELDS if sha(getattr(res, f)) != g[f]["sha256"]]
    sums = {f: (int(getattr(res, f).astype(np.uint64).sum(dtype=np.uint64)), g[f]["sum"]) for f in bad}
    assert not bad, f"{name}: arrays differ from the oracle: {sums}"


def _trace(name):
    tr = trace_of(name)
    assert trace_hash(tr) == GOLD[name]["trace_sha256"], "synthetic trace generator changed"
    return tr


@pytest.mark.parametrize("lookback", ["0", "1"])
@pytest.mark.parametrize("name", ["32x32_uniform_l0.005_ppt10000", "32x32_hotspot_l0.005_ppt10000"])
def test_configs1_full_size_matches_oracle(name, lookback, monkeypatch):
    """Both chain hand-off protocols (GNOC_CHAIN_LOOKBACK: 0 serial, 1 look-back), over
    several runs so the adapted windows (and their spill patterns) are covered too."""
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", lookback)
    tr = _trace(name)
    cfg = gnoc.EngineConfig(num_tiles=1024)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    for k in range(3):
        eng.run()
        s = eng.summary()
        assert s["engine_path"] == 4 and s["fallbacks"] == 0
        assert s["mesh_hops"] == GOLD[name]["mesh_hops"]
        _check(name, eng.results())
    eng.close()


@pytest.mark.parametrize("lookback", ["0", "1"])
def test_configs1_full_size_mg1_burst_matches_oracle(lookback, monkeypatch):
    """configs[1]'s uniform batch behind a cycle-0 burst (4 packets per tile): the
    analytical M/G/1 branch serves requests in injection and mesh ports, so the
    pin covers mg1_uses > 0 at full size.  Every result array hashes as the
    oracle's and the summary's M/G/1 count equals the oracle's; the engine path
    each run took is printed (the chains run the no-gap M/G/1 prefix serially or
    the batch takes a slower exact path; the bench reports which)."""
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", lookback)
    name = "32x32_burst4_l0.005_ppt10000"
    assert GOLD[name]["mg1_uses"] > 0
    assert GOLD[name]["results"]["port_mg1"]["sum"] == GOLD[name]["mg1_uses"]
    tr = _trace(name)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
    eng.submit(tr)
    paths = []
    for r in range(5):
        eng.run()
        s = eng.summary()
        paths.append(int(s["engine_path"]))
        assert s["mg1_uses"] == GOLD[name]["mg1_uses"], (s["mg1_uses"], GOLD[name]["mg1_uses"])
        _check(name, eng.results())
        if r:   # later runs go straight to k_chain's MG instantiation (bit 10) ...
            assert s["engine_path"] == 4 and s["chain_protocol"] & 0x400, s
            assert s["retries"] == 0 and s["fallbacks"] == 0, s
    # ... and once the windows have settled and its M/G/1 windows are known, only those
    # take the M/G/1 path (bit 11, k_chain_mix)
    assert s["chain_protocol"] & 0x800, s
    eng.close()
    print("engine paths", paths)


def test_configs1_full_size_level_engine_matches_oracle(monkeypatch):
    """The chunked level engine (the chain engine's fallback) on the same batch."""
    name = "32x32_uniform_l0.005_ppt10000"
    monkeypatch.setenv("GNOC_ENGINE", "levels")
    tr = _trace(name)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
    eng.submit(tr)
    eng.run()
    assert eng.summary()["engine_path"] == 1
    res = eng.results()
    eng.close()
    _check(name, res)


@pytest.mark.parametrize("lookback", ["0", "1"])
def test_configs2_full_size_matches_oracle_single_and_8_ranks(lookback, monkeypatch):
    monkeypatch.setenv("GNOC_CHAIN_LOOKBACK", lookback)
    name = "64x64_uniform_l0.002_ppt10000"
    tr = _trace(name)
    cfg = gnoc.EngineConfig(num_tiles=4096)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    res = eng.results()
    eng.close()
    _check(name, res)
    ss = gnoc.LocalShardSet(cfg, 8)
    ss.submit(tr)
    ss.run()
    got = ss.results()
    ss.close()
    _check(name, got)
