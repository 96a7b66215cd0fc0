"""GPU engine vs CPU oracle: bit-exact per-packet times and per-port counters.

Integer/ps arithmetic, so the bar is exact equality (np.array_equal) on every
output array.  Runs on the MI355X box through the C ABI (libgnoc.so).
"""
import os

import numpy as np
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.traces import random_trace

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def run_both(cfg, tr):
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    got = eng.results()
    eng.close()
    ref = oracle.run(cfg, tr)
    return got, ref


def assert_same(got, ref, tr=None):
    for name in ("final_ps", "zero_load_ps", "contention_ps"):
        a, b = getattr(got, name), getattr(ref, name)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            raise AssertionError(f"{name}: {bad.size} mismatches, first id {bad[0]}: gpu {a[bad[0]]} oracle {b[bad[0]]}")
    for name in ("port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
        a, b = getattr(got, name), getattr(ref, name)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0]
            raise AssertionError(f"{name}: {bad.size} ports differ, first port {bad[0]}: gpu {a[bad[0]]} oracle {b[bad[0]]}")


@pytest.mark.parametrize("load,ppt", [(0.02, 300), (0.05, 300), (0.3, 100)])
def test_synthetic_8x8(load, ppt):
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, load, ppt, seed=11)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)
    assert got.summary["mesh_hops"] == int(ref.port_count.reshape(-1, 6)[:, :5].sum())


def test_declined_batch_reruns_identically():
    """A batch the chain engine declines (saturated bursts: the M/G/1 branch
    fires) runs on the level engine; later runs of the same batch go there
    directly (no doomed attempt) and give the same bytes."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(6000, 8, 8, seed=21, max_cycle=150, burst0=200)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    a, s1 = eng.results(), eng.summary()
    eng.run()
    b, s2 = eng.results(), eng.summary()
    eng.close()
    assert s1["fallbacks"] >= 1 and s2["fallbacks"] == 0 and s1["engine_path"] == s2["engine_path"] != 4
    assert_same(a, b)
    assert_same(a, oracle.run(cfg, tr))


def test_saturated_mg1_is_exercised():
    """Saturated 8x8 from t=0: the M/G/1 fallback fires and must match."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(20000, 8, 8, seed=3, max_cycle=300, burst0=400)
    got, ref = run_both(cfg, tr)
    assert ref.port_mg1.sum() > 0
    assert_same(got, ref)


@pytest.mark.parametrize("W,H", [(4, 4), (2, 4), (3, 3), (1, 5), (6, 6)])
def test_mesh_shapes_and_bursts(W, H):
    cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H)
    tr = random_trace(3000, W, H, seed=W * 10 + H, max_cycle=400, burst0=50, self_frac=0.05)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


def test_self_and_unmodeled_bypass():
    cfg = gnoc.EngineConfig(num_tiles=16)
    tr = random_trace(4000, 4, 4, seed=5, max_cycle=500, self_frac=0.2, unmodeled_frac=0.2)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)
    selfm = tr.src == tr.dst
    assert np.array_equal(got.final_ps[selfm], tr.inject_ps[selfm])


@pytest.mark.parametrize("flit_width", [16, 32, 128])
@pytest.mark.parametrize("router_delay", [0, 2])
def test_flit_width_router_delay(flit_width, router_delay):
    cfg = gnoc.EngineConfig(num_tiles=36, flit_width=flit_width, router_delay=router_delay)
    tr = random_trace(5000, 6, 6, seed=flit_width + router_delay, max_cycle=2000, burst0=20,
                      bits_choices=[72, 576, 584, 1088])
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


def test_link_delay_two():
    # tile_width 150 mm at 1 GHz -> ceil(1.5) = 2-cycle links (electrical_link_model.cc:13-16)
    cfg = gnoc.EngineConfig(num_tiles=16, tile_width_mm=150.0, link_delay=2)
    tr = random_trace(4000, 4, 4, seed=9, max_cycle=600, burst0=10)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


@pytest.mark.parametrize("freq", [0.9, 1.5, 0.7])
def test_non_unit_frequency(freq):
    import math
    lk = math.ceil(freq * 0.01 * 1.0)
    cfg = gnoc.EngineConfig(num_tiles=16, frequency_ghz=freq, link_delay=lk)
    tr = random_trace(3000, 4, 4, seed=int(freq * 10), max_cycle=500, burst0=8, ps_jitter=True,
                      frequency_ghz=freq)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    got = eng.results()
    assert eng.summary()["engine_path"] in (1, 4)   # chunked or chain kernels with the double ps <-> cycle conversions
    eng.close()
    assert_same(got, oracle.run(cfg, tr))


@pytest.mark.parametrize("freq", [0.9, 1.25, 0.7, 1.5])
def test_non_unit_frequency_chain_engine(freq):
    """f != 1 GHz on the chain engine (Time::toCycles / Latency::toPicosec, time_types.h:81-109,
    as the reference's double expressions): a 16x16 synthetic batch stays on engine path 4
    and is bit-exact, ports included."""
    cfg = gnoc.EngineConfig(num_tiles=256, frequency_ghz=freq)
    tr = gnoc.synthetic_trace(16, 16, 0.01, 300, seed=int(freq * 100), frequency_ghz=freq)
    got, ref = run_both(cfg, tr)
    assert got.summary["engine_path"] == 4 and got.summary["fallbacks"] == 0
    assert_same(got, ref)
    for k in ("port_flit", "port_last"):
        assert np.array_equal(getattr(got, k), getattr(ref, k)), k


@pytest.mark.parametrize("freq", [0.9, 1.25])
def test_non_unit_frequency_chunked_8x8(freq):
    """f != 1 GHz on the chunked path at a size with many chunks per port,
    M/G/1 bursts included (Time::toCycles / Latency::toPicosec, time_types.h:81-109)."""
    cfg = gnoc.EngineConfig(num_tiles=64, frequency_ghz=freq)
    tr = random_trace(40000, 8, 8, seed=int(freq * 100), max_cycle=4000, burst0=300, frequency_ghz=freq)
    got, ref = run_both(cfg, tr)
    assert ref.port_mg1.sum() > 0
    assert_same(got, ref)
    for k in ("port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
        assert np.array_equal(getattr(got, k), getattr(ref, k)), k


@pytest.mark.parametrize("max_list,analytical", [(2, 1), (3, 1), (100, 0), (5, 1)])
def test_queue_parameters(max_list, analytical):
    cfg = gnoc.EngineConfig(num_tiles=16, max_list_size=max_list, analytical_enabled=bool(analytical))
    tr = random_trace(3000, 4, 4, seed=max_list * 7 + analytical, max_cycle=300, burst0=30)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


def test_contention_disabled():
    cfg = gnoc.EngineConfig(num_tiles=64, contention_enabled=False)
    tr = gnoc.synthetic_trace(8, 8, 0.1, 100, seed=2)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)
    assert got.contention_ps.max() == 0


def test_empty_and_single():
    cfg = gnoc.EngineConfig(num_tiles=16)
    tr = random_trace(0, 4, 4)
    got, ref = run_both(cfg, tr)
    assert got.final_ps.size == 0
    tr = random_trace(1, 4, 4, seed=1)
    tr.src[:] = 0
    tr.dst[:] = 15
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)
    # zero-load closed form: (H+1)(R+Lk) + F = 7*2 + 9
    assert int(got.final_ps[0] - tr.inject_ps[0]) == (7 * 2 + 9) * 1000


def test_hotspot_32x32():
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.005, 40, seed=4, hotspot_fraction=0.2, num_hotspots=16)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


def test_uniform_32x32():
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.01, 60, seed=5)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


def test_repeatable_bytes():
    """Deterministic by construction: the same batch twice gives identical bytes."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, 0.08, 200, seed=13)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    a = eng.results()
    eng.run()
    b = eng.results()
    assert np.array_equal(a.final_ps, b.final_ps) and np.array_equal(a.port_sum_delay, b.port_sum_delay)


def test_serial_prefix_spans_chunks():
    """A 3000-packet burst at t=0 from one tile keeps its injection queue in the
    history-tree/M-G-1 serial prefix across several chunks (look-back must hand
    over the serial state), and floods one row (burst splitting)."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(12000, 8, 8, seed=21, max_cycle=4000)
    tr.inject_ps[:3000] = 0
    tr.src[:3000] = 9
    order = np.lexsort((np.arange(len(tr)), tr.inject_ps))
    tr = type(tr)(tr.inject_ps[order], tr.src[order], tr.dst[order], tr.bits[order], tr.flags[order])
    got, ref = run_both(cfg, tr)
    assert ref.port_mg1.sum() > 1000
    assert_same(got, ref)


def test_bursty_input_splits_leaves():
    """Bursts on one input of a port (many packets at the same cycle from one
    tile towards one column) force the chunk splitter to cut leaves."""
    cfg = gnoc.EngineConfig(num_tiles=256, analytical_enabled=False)
    rng = np.random.default_rng(3)
    n = 60000
    t = np.sort(rng.integers(0, 20000, n)).astype(np.uint64) * np.uint64(1000)
    src = rng.integers(0, 256, n).astype(np.uint32)
    dst = rng.integers(0, 256, n).astype(np.uint32)
    burst = (t // 1000) % 2000 < 30
    src[burst] = 16 * 5 + 1
    dst[burst] = 16 * 12 + 14
    tr = gnoc.Trace(t, src, dst, np.full(n, 576, np.uint32), np.zeros(n, np.uint32))
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


def test_engine_paths_agree():
    """Whole-port streams (v1) and chunked look-back (v2) give identical bytes."""
    import os
    cfg = gnoc.EngineConfig(num_tiles=256)
    tr = gnoc.synthetic_trace(16, 16, 0.02, 200, seed=8)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    a = eng.results()
    assert a.summary["engine_path"] == 1
    os.environ["GNOC_ENGINE"] = "v1"
    try:
        eng.run()
        b = eng.results()
    finally:
        del os.environ["GNOC_ENGINE"]
    assert b.summary["engine_path"] == 0
    for k in ("final_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


@pytest.mark.parametrize("chunk", [64, 200, 400, 800])
def test_small_chunks_serial_prefix_and_exception_tails(chunk, monkeypatch):
    """GNOC_CHUNK cuts every port into many chunks: the history tree's serial
    (M/G/1) prefix, and M/G/1 exception tails whose keys fall before a port's
    first FIFO record, cross chunk boundaries -- including an empty chunk 0 that
    must hand the untouched serial state to its successor."""
    monkeypatch.setenv("GNOC_CHUNK", str(chunk))
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(20000, 8, 8, seed=3, max_cycle=300, burst0=400)
    got, ref = run_both(cfg, tr)
    assert ref.port_mg1.sum() > 0
    assert_same(got, ref)


@pytest.mark.parametrize("chunk", [128, 512])
def test_small_chunks_32x32_hotspot(chunk, monkeypatch):
    monkeypatch.setenv("GNOC_CHUNK", str(chunk))
    cfg = gnoc.EngineConfig(num_tiles=1024)
    tr = gnoc.synthetic_trace(32, 32, 0.01, 100, seed=8, hotspot_fraction=0.2, num_hotspots=16)
    got, ref = run_both(cfg, tr)
    assert_same(got, ref)


@pytest.mark.parametrize("qtype,L,inter", [(gnoc.QUEUE_BASIC, 100, True), (gnoc.QUEUE_HISTORY_LIST, 2, True),
                                           (gnoc.QUEUE_HISTORY_LIST, 3, False), (gnoc.QUEUE_HISTORY_LIST, 100, True)])
def test_queue_models_basic_and_history_list(qtype, L, inter):
    """QueueModel::create's other types (queue_model.cc:18-38) against the
    oracle's restatements of queue_model_basic.cc / queue_model_history_list.cc."""
    cfg = gnoc.EngineConfig(num_tiles=64, queue_type=qtype, max_list_size=L, interleaving_enabled=inter)
    tr = random_trace(20000, 8, 8, seed=3, max_cycle=300, burst0=400)
    got, ref = run_both(cfg, tr)
    if qtype == gnoc.QUEUE_HISTORY_LIST:
        assert ref.port_mg1.sum() > 0
    else:
        assert ref.port_mg1.sum() == 0
    assert_same(got, ref)


@pytest.mark.parametrize("N,R,f", [(64, 1, 1.0), (12, 0, 1.0), (10, 2, 0.9), (1024, 3, 1.5)])
def test_emesh_hop_counter_model(N, R, f):
    """NetworkModelEMeshHopCounter (network_model_emesh_hop_counter.cc:143-157):
    the contention-free model, including non-rectangular tile counts."""
    import math
    cfg = gnoc.EngineConfig(num_tiles=N, router_delay=R, frequency_ghz=f)
    w = int(math.floor(math.sqrt(N)))
    tr = random_trace(3000, w, int(math.ceil(N / w)), seed=N + R, max_cycle=500, self_frac=0.05, unmodeled_frac=0.05,
                      bits_choices=[72, 576, 1088], frequency_ghz=f)
    ok = (tr.src < N) & (tr.dst < N)
    tr = gnoc.Trace(tr.inject_ps[ok], tr.src[ok], tr.dst[ok], tr.bits[ok], tr.flags[ok])
    eng = gnoc.Engine(cfg, model="emesh_hop_counter")
    eng.submit(tr)
    eng.run()
    got = eng.results()
    eng.close()
    ref = oracle.run_hop_counter(cfg, tr)
    for k in ("final_ps", "zero_load_ps", "contention_ps"):
        assert np.array_equal(getattr(got, k), getattr(ref, k)), k


AM, GM, MED = gnoc.MOVING_AVG_ARITHMETIC_MEAN, gnoc.MOVING_AVG_GEOMETRIC_MEAN, gnoc.MOVING_AVG_MEDIAN


@pytest.mark.parametrize("ma,w,t0", [(AM, 64, 0), (AM, 1, 0), (AM, 5, 0), (MED, 64, 0), (MED, 4, 0), (MED, 1, 0),
                                     (GM, 64, 0), (GM, 1, 0), (GM, 5, 0), (GM, 64, 1), (GM, 7, 1), (GM, 200, 1),
                                     (AM, 64, 2), (MED, 4, 2), (GM, 16, 2)])
def test_basic_moving_average(ma, w, t0):
    """QueueModelBasic with moving_avg_enabled (queue_model_basic.cc:7-61,
    moving_average.h; carbon_sim.cfg:376-379 default = arithmetic_mean over 64):
    engine path 3 bit-exact against the oracle, whose moving averages are pinned
    against the reference's own moving_average.h (tests/test_oracle.py).
    The geometric mean runs glibc's pow (glibc_pow.h).  t0 = 0: packets at cycle
    0 put zeros into the windows (the geometric mean becomes 0, then NaN once a
    zero leaves the window: ref = (UInt64) NaN as on x86-64); t0 = 1: every
    request at cycle >= 1000, so the products stay finite; t0 = 2: times beyond
    2^33 ps (the 49-bit sort keys instead of 32-bit ones)."""
    cfg = gnoc.EngineConfig(num_tiles=64, queue_type=gnoc.QUEUE_BASIC, moving_avg_type=ma, moving_avg_window=w)
    tr = random_trace(20000, 8, 8, seed=w + 7 * ma, max_cycle=2000, burst0=300, self_frac=0.03, unmodeled_frac=0.03,
                      bits_choices=[72, 576, 1088])
    if t0:
        tr.inject_ps[:] += 1_000_000 if t0 == 1 else (1 << 33)
    got, ref = run_both(cfg, tr)
    assert got.summary["engine_path"] == 3
    assert_same(got, ref)


@pytest.mark.parametrize("W,H,f,load,ma", [(32, 32, 1.0, 0.005, AM), (5, 3, 0.9, 0.05, AM), (1, 6, 1.0, 0.05, AM),
                                           (6, 1, 1.5, 0.05, AM), (32, 32, 1.0, 0.005, GM), (5, 3, 0.9, 0.05, GM),
                                           (6, 1, 1.5, 0.05, GM), (32, 32, 1.0, 0.005, MED)])
def test_basic_moving_average_meshes(W, H, f, load, ma):
    """Moving-average basic queues on a 32x32 synthetic batch (configs[1]'s
    traffic, 100 packets per tile), odd and one-wide meshes and f != 1 GHz.
    At 32x32 the geometric mean's pow(mean, 63) overflows to inf for cycle
    counts above ~8e4 (moving_average.h:129), as in the reference."""
    cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H, frequency_ghz=f,
                            queue_type=gnoc.QUEUE_BASIC, moving_avg_type=ma)
    if W == H:
        tr = gnoc.synthetic_trace(W, H, load, 100, seed=5)
    else:
        tr = random_trace(6000, W, H, seed=W * 10 + H, max_cycle=1500, burst0=50, frequency_ghz=f,
                          ps_jitter=True)
    got, ref = run_both(cfg, tr)
    assert got.summary["engine_path"] == 3
    assert_same(got, ref)


def test_basic_moving_average_refusals():
    """Broadcast batches, sharding and non-basic queues are refused, not
    approximated."""
    cfg = gnoc.EngineConfig(num_tiles=16, queue_type=gnoc.QUEUE_BASIC, moving_avg_type=gnoc.MOVING_AVG_MEDIAN)
    eng = gnoc.Engine(cfg)
    tr = random_trace(200, 4, 4, seed=1, bcast_frac=0.1)
    eng.submit(tr)
    with pytest.raises(gnoc.GnocError) as ex:
        eng.run()
    assert ex.value.code == -5
    with pytest.raises(gnoc.GnocError) as ex:
        eng._check(eng.lib.gnoc_shard(eng._h, 0, 2))
    assert ex.value.code == -5
    eng.close()
    with pytest.raises(gnoc.GnocError) as ex:
        gnoc.Engine(gnoc.EngineConfig(num_tiles=16, moving_avg_type=gnoc.MOVING_AVG_MEDIAN))
    assert ex.value.code == -1


@pytest.mark.parametrize("name", sorted(f[:-4] for f in os.listdir(GOLD) if f.endswith(".npz")))
def test_engine_matches_golden_fixtures(name):
    """The engine against every committed golden fixture (tests/golden/*.npz,
    produced by make_golden.py from the pinned oracle): packets and port counters."""
    import json
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    cfg = gnoc.EngineConfig(**json.loads(str(z["cfg"])))
    tr = gnoc.Trace(z["inject_ps"], z["src"], z["dst"], z["bits"], z["flags"])
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    got = eng.results()
    eng.close()
    for k in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1"):
        assert np.array_equal(getattr(got, k), z[k]), k
