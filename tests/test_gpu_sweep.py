"""Design-space sweep (gnoc_create_sweep): many points with their own flit
width, router delay and link delay in one batch, each bit-exact against the
oracle run of that point alone."""
import itertools

import numpy as np
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.traces import random_trace

pytestmark = pytest.mark.gpu


def check_points(base, pts, traces):
    eng = gnoc.SweepEngine(base, pts)
    eng.submit(traces)
    eng.run()
    eng.run()
    got = eng.results()
    eng.close()
    for k, (q, tr) in enumerate(zip(pts, traces)):
        ref = oracle.run(q.config(base), tr)
        for name in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
            a, b = getattr(got[k], name), getattr(ref, name)
            assert np.array_equal(a, b), f"point {k} {q}: {name} differs ({np.sum(a != b)} entries)"


def test_sweep_grid_of_config5_axes():
    """flit width x router delay x tile width (-> link delay 1..4) x load, 8x8 points."""
    base = gnoc.EngineConfig(num_tiles=64)
    pts, trs = [], []
    axes = itertools.product([16, 32, 64, 128], [0, 1, 2, 3], [1.0, 150.0, 250.0, 350.0])
    for k, (fw, r, tw) in enumerate(axes):
        if k % 3:
            continue   # 22 of the 64 combinations keep the test short
        lk = int(np.ceil(0.01 * tw))
        pts.append(gnoc.SweepPoint(fw, r, lk, tw))
        load = (0.005, 0.01, 0.015, 0.02)[k % 4]
        trs.append(gnoc.synthetic_trace(8, 8, load, 150, seed=100 + k))
    check_points(base, pts, trs)


def test_sweep_saturated_points_with_mg1():
    base = gnoc.EngineConfig(num_tiles=16)
    pts = [gnoc.SweepPoint(64, 1, 1, 1.0), gnoc.SweepPoint(16, 2, 2, 150.0), gnoc.SweepPoint(128, 0, 3, 250.0)]
    trs = [random_trace(3000, 4, 4, seed=s, max_cycle=200, burst0=100, self_frac=0.05) for s in range(3)]
    check_points(base, pts, trs)
    assert sum(oracle.run(q.config(base), t).port_mg1.sum() for q, t in zip(pts, trs)) > 0


def test_sweep_one_point_is_the_plain_engine():
    base = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, 0.02, 300, seed=1)
    check_points(base, [gnoc.SweepPoint()], [tr])


def test_sweep_256_points_full_grid():
    """All 256 points of SURVEY 8d config 5 in one batch (a 128 x 128 block
    mesh: the large-mesh scatter and multi-block slot scan), light traffic."""
    base = gnoc.EngineConfig(num_tiles=64)
    pts, trs = [], []
    for k, (fw, r, tw, load) in enumerate(itertools.product([16, 32, 64, 128], [0, 1, 2, 3],
                                                            [1.0, 150.0, 250.0, 350.0], [0.005, 0.01, 0.015, 0.02])):
        pts.append(gnoc.SweepPoint(fw, r, int(np.ceil(0.01 * tw)), tw))
        trs.append(gnoc.synthetic_trace(8, 8, load, 12, seed=1000 + k))
    check_points(base, pts, trs)


def test_sweep_256_points_benched_length_pinned():
    """BASELINE.json configs[4] at the length bench.py times it: all 256 points at
    2,000 packets per tile (bench.py's seeds), one batch, every point's eight result
    arrays against the oracle's SHA-256 (tests/golden/make_sweep.py).  The saturated
    points' long queues and M/G/1 requests are exercised here at full length."""
    import json
    import os
    from tests.golden import make_sweep as ms
    with open(os.path.join(os.path.dirname(__file__), "golden", "sweep_hashes.json")) as fh:
        gold = json.load(fh)
    pts = ms.points()
    trs = [ms.trace(i, load) for i, (_, load) in enumerate(pts)]
    for i in (0, 127, 255):
        assert ms.trace_hash(trs[i]) == gold["points"][i]["trace_sha256"], "sweep trace generator changed"
    eng = gnoc.SweepEngine(gnoc.EngineConfig(num_tiles=64), [q for q, _ in pts])
    eng.submit(trs)
    for _ in range(2):
        eng.run()
        got = eng.results()
        bad = [i for i in range(len(pts)) if ms.point_hash(got[i]) != gold["points"][i]["hash"]]
        assert not bad, f"{len(bad)} points differ from the oracle, first {bad[0]}: {pts[bad[0]]}"
    print("sweep engine path", eng.summary()["engine_path"], "mg1 uses", sum(p["mg1_uses"] for p in gold["points"]))
    eng.close()
