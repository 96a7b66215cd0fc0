"""BASELINE.json workloads at full size, checked through size-independent
properties (the oracle would take minutes here; it pins the small cases):

* the closed form: final = inject + zero_load + contention, zero_load =
  (H+1)(R+Lk) + F cycles, per packet;
* a checksum of checksums: the per-port contention sums equal the per-packet
  contention delays summed (every cycle of contention is charged to exactly one
  port, router_model.cc:136-144), and the per-port request counts equal the
  route lengths;
* determinism: a second run gives identical bytes;
* sharding: 8 row/column-band ranks give the unsharded 64x64 results exactly.
"""
import numpy as np
import pytest

from graphite_amd import gnoc

pytestmark = pytest.mark.gpu


def _route_len(tr, W):
    sx, sy = tr.src % W, tr.src // W
    dx, dy = tr.dst % W, tr.dst // W
    return np.abs(sx.astype(np.int64) - dx) + np.abs(sy.astype(np.int64) - dy)


def _check_properties(cfg, tr, r):
    W = cfg.width
    routed = (tr.src != tr.dst)
    H = _route_len(tr, W)
    F = (tr.bits.astype(np.int64) + cfg.flit_width - 1) // cfg.flit_width
    rl = (cfg.router_delay + cfg.link_delay) * 1000
    zl = np.where(routed, (H + 1) * rl + F * 1000, 0)
    assert np.array_equal(r.zero_load_ps.astype(np.int64), zl)
    assert np.array_equal(r.final_ps, tr.inject_ps + r.zero_load_ps + r.contention_ps)
    assert int(r.port_sum_delay.sum()) * 1000 == int(r.contention_ps.astype(np.int64).sum())
    pc = r.port_count.reshape(-1, 6)
    assert int(pc[:, :5].sum()) == int((H + 1)[routed].sum())          # mesh routers
    assert int(pc[:, 5].sum()) == int(routed.sum())                     # injection routers
    # per-port flits: every request's F (queue_model.cc:49-53)
    assert int(r.port_flit.sum()) == int((F * (H + 2))[routed].sum())


@pytest.mark.parametrize("mix", ["uniform", "hotspot"])
def test_32x32_baseline_config_properties(mix):
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.005, 10000, seed=1, hotspot_fraction=0.2 if mix == "hotspot" else 0.0,
                              num_hotspots=16)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    a = eng.results()
    eng.run()
    b = eng.results()
    eng.close()
    _check_properties(cfg, tr, a)
    for k in ("final_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


def test_64x64_sharded_8_ranks_equals_unsharded():
    cfg = gnoc.EngineConfig(num_tiles=4096)
    tr = gnoc.synthetic_trace(64, 64, 0.002, 10000, seed=1)
    e = gnoc.Engine(cfg)
    e.submit(tr)
    e.run()
    ref = e.results()
    e.close()
    _check_properties(cfg, tr, ref)
    ss = gnoc.LocalShardSet(cfg, 8)
    ss.submit(tr)
    ss.run()
    got = ss.results()
    ss.close()
    for k in ("final_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
        assert np.array_equal(getattr(got, k), getattr(ref, k)), k
