"""The delta wire format's host encoder (include/gnoc.h gnoc_pack_trace, the
library's threads) against the numpy restatement of the same format
(PackedTrace.of_numpy): identical arrays on traces with and without escapes,
varying lengths, flags, ties and empty batches; fields that do not fit are refused."""
import numpy as np
import pytest

from graphite_amd import gnoc
from tests.traces import random_trace


def _same(a, b):
    assert a.t0 == b.t0 and a.bits_all == b.bits_all
    for k in ("dt", "abs_ps", "src", "dst"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    for k in ("bits", "flags"):
        x, y = getattr(a, k), getattr(b, k)
        assert (x is None) == (y is None), k
        if x is not None:
            np.testing.assert_array_equal(x, y, err_msg=k)


@pytest.mark.parametrize("case", ["synthetic", "jitter", "bits", "flags", "gaps", "empty", "one"])
def test_encoder_matches_numpy(case):
    if case == "synthetic":
        tr = gnoc.synthetic_trace(32, 32, 0.005, 300, seed=3)
    elif case == "jitter":
        tr = random_trace(200000, 8, 8, seed=4, max_cycle=30000, ps_jitter=True)
    elif case == "bits":
        tr = random_trace(150000, 8, 8, seed=5, max_cycle=20000, bits_choices=[64, 576, 1024])
    elif case == "flags":
        tr = random_trace(150000, 6, 6, seed=6, max_cycle=20000, unmodeled_frac=0.2)
    elif case == "gaps":
        rng = np.random.default_rng(7)
        t = np.cumsum(rng.choice([0, 1000, 70000, 1 << 40], 300000, p=[0.3, 0.5, 0.19, 0.01])).astype(np.uint64)
        tr = gnoc.Trace(t, rng.integers(0, 64, t.size).astype(np.uint32), rng.integers(0, 64, t.size).astype(np.uint32),
                        np.full(t.size, 576, np.uint32), np.zeros(t.size, np.uint32))
    elif case == "empty":
        tr = gnoc.Trace(np.zeros(0, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32),
                        np.zeros(0, np.uint32))
    else:
        tr = gnoc.Trace(np.array([5_000_000], np.uint64), np.array([3], np.uint32), np.array([9], np.uint32),
                        np.array([200], np.uint32), np.zeros(1, np.uint32))
    got, ref = gnoc.PackedTrace.of(tr), gnoc.PackedTrace.of_numpy(tr)
    _same(got, ref)
    assert got.wire_bytes() == ref.wire_bytes()


def test_encoder_refuses_wide_fields():
    tr = gnoc.synthetic_trace(8, 8, 0.01, 50, seed=1)
    tr.bits[7] = 1 << 16
    with pytest.raises(ValueError):
        gnoc.PackedTrace.of(tr)
    with pytest.raises(ValueError):
        gnoc.PackedTrace.of_numpy(tr)
