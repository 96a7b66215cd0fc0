"""The submit contract (include/gnoc.h gnoc_submit / gnoc_submit_device),
checked on the device by prep.hip k_validate for both entry points: a bad trace
is refused with GNOC_ETRACE / GNOC_EUNSUPPORTED naming the first offending
packet, never run; a trace already in HBM runs like the same trace from the
host (both on the chain engine, windows sized from the device statistics)."""
import numpy as np
import pytest

from graphite_amd import gnoc
from tests.traces import random_trace

pytestmark = pytest.mark.gpu

ETRACE, EUNSUPPORTED, ESTATE = -2, -5, -4


def _device_submit(eng, tr):
    import torch
    tr = tr.normalized()
    dev = torch.device("cuda", 0)
    ts = [torch.from_numpy(a.view(np.int64 if a.dtype == np.uint64 else np.int32).copy()).to(dev)
          for a in (tr.inject_ps, tr.src, tr.dst, tr.bits, tr.flags)]
    torch.cuda.synchronize()
    eng.submit_device(*(t.data_ptr() for t in ts), len(tr), keep=ts)


def _bad(kind):
    tr = random_trace(400, 4, 4, seed=3, max_cycle=300)
    if kind == "tile":
        tr.src[5] = 16
        return tr, ETRACE, "packet 5"
    if kind == "order":
        tr.inject_ps[7] = tr.inject_ps[8] + 1000   # packet 8 arrives before packet 7
        return tr, ETRACE, "packet 8"
    if kind == "zero":
        i = int(np.nonzero(tr.src != tr.dst)[0][0])
        tr.bits[i] = 0
        return tr, ETRACE, f"packet {i}"
    if kind == "fmax":
        tr.bits[11] = 64 * 2048
        return tr, EUNSUPPORTED, "packet 11"
    if kind == "first":
        # two violations: the lower packet index is the one reported
        tr.src[90] = 99
        tr.inject_ps[40] = tr.inject_ps[41] + 5000
        return tr, ETRACE, "not ordered"
    raise ValueError(kind)


@pytest.mark.parametrize("path", ["host", "device"])
@pytest.mark.parametrize("kind", ["tile", "order", "zero", "fmax", "first"])
def test_bad_trace_refused(path, kind):
    tr, code, text = _bad(kind)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=16))
    try:
        with pytest.raises(gnoc.GnocError) as ex:
            if path == "host":
                eng.submit(tr)
            else:
                _device_submit(eng, tr)
        assert ex.value.code == code
        assert text in str(ex.value) or text in eng.lib.gnoc_last_error(eng._h).decode()
        # a refused trace is not runnable
        with pytest.raises(gnoc.GnocError) as ex2:
            eng.run()
        assert ex2.value.code == ESTATE
    finally:
        eng.close()


def test_device_resident_trace_matches_host_submit():
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, 0.02, 300, seed=11)
    a = gnoc.Engine(cfg)
    a.submit(tr)
    a.run()
    ra, sa = a.results(), a.summary()
    a.close()
    b = gnoc.Engine(cfg)
    _device_submit(b, tr)
    b.run()
    rb, sb = b.results(), b.summary()
    b.close()
    assert sa["engine_path"] == sb["engine_path"] == 4
    assert sa["windows"] == sb["windows"]
    for f in ("final_ps", "contention_ps", "port_sum_delay", "port_count", "port_flit", "port_last"):
        assert np.array_equal(getattr(ra, f), getattr(rb, f)), f


@pytest.mark.parametrize("bound", ["1", "3000"])
def test_slot_layout_past_the_record_bound_is_refused(bound, monkeypatch):
    """The slot-layout guard (prep.hip k_scan_slots): a layout that would reach past
    the record buffer (here: the bound lowered by GNOC_TEST_LAYOUT_BOUND, below the
    mesh slots or below even the injection slots) empties the mesh slots, so no
    later kernel writes outside the buffer, and the run is refused.  The engine
    then runs the batch exactly with the bound restored."""
    from oracle import oracle
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, 0.02, 300, seed=5)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    monkeypatch.setenv("GNOC_TEST_LAYOUT_BOUND", bound)
    with pytest.raises(gnoc.GnocError, match="record bound"):
        eng.run()
    monkeypatch.delenv("GNOC_TEST_LAYOUT_BOUND")
    eng.run()
    np.testing.assert_array_equal(eng.results().final_ps, oracle.run(cfg, tr).final_ps)
    eng.close()
