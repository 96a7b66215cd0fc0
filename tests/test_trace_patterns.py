"""Destinations of the synthetic traffic patterns (gnoc_trace_synthetic_pattern)
against the reference generator's formulas (synthetic_network.cc:288-341),
restated here independently; the timing model is the uniform case's."""
import numpy as np
import pytest

from graphite_amd import gnoc


def _expected(pattern, W, H, t):
    N = W * H
    sx, sy = t % W, t // W
    nbits = int(np.log2(N))
    return {
        "bit_complement": (~t) & (N - 1),
        "shuffle": ((t >> (nbits - 1)) & 1) | ((t << 1) & (N - 1)),
        "transpose": sx * W + sy,
        "tornado": ((sy + H // 2) % H) * W + (sx + W // 2) % W,
        "nearest_neighbor": ((sy + 1) % H) * W + (sx + 1) % W,
    }[pattern]


@pytest.mark.parametrize("pattern", ["bit_complement", "shuffle", "transpose", "tornado", "nearest_neighbor"])
@pytest.mark.parametrize("W,H", [(8, 8), (32, 32), (16, 16)])
def test_pattern_destinations(pattern, W, H):
    tr = gnoc.synthetic_trace(W, H, 0.05, 20, seed=2, pattern=pattern)
    assert len(tr) == W * H * 20
    assert np.all(np.diff(tr.inject_ps.astype(np.int64)) >= 0)
    exp = np.array([_expected(pattern, W, H, t) for t in range(W * H)], np.uint32)
    assert np.array_equal(tr.dst, exp[tr.src])
    # the same per-tile send times as uniform traffic (the Bernoulli stream is the tile's)
    u = gnoc.synthetic_trace(W, H, 0.05, 20, seed=2)
    assert np.array_equal(np.sort(u.inject_ps), np.sort(tr.inject_ps))


def test_pattern_refusals():
    # bit complement / shuffle need 2^k tiles (the reference asserts isPower2)
    for p in ("bit_complement", "shuffle"):
        with pytest.raises(gnoc.GnocError) as ex:
            gnoc.synthetic_trace(6, 6, 0.05, 5, pattern=p)
        assert ex.value.code == -1
    with pytest.raises(ValueError):
        gnoc.synthetic_trace(4, 4, 0.05, 5, pattern="hotspot_storm")


def test_packed_wire_format_round_trip_on_host():
    """gnoc.PackedTrace (gnoc_packets_packed): the u16 differences with 0xFFFF escapes
    to absolute times restate the inject times exactly (host decode of the format the
    device scan decodes); one-length batches drop the length array."""
    import numpy as np
    from graphite_amd import gnoc
    tr = gnoc.synthetic_trace(8, 8, 0.02, 500, seed=3).normalized()
    t = tr.inject_ps.astype(np.uint64)
    t[100:] += np.uint64(1 << 40)
    t[101:] += np.uint64(65_535)
    tr = gnoc.Trace(t, tr.src, tr.dst, tr.bits, tr.flags)
    pt = gnoc.PackedTrace.of(tr)
    assert pt.bits is None and pt.flags is None and pt.abs_ps.size >= 2
    out, T, k = [], pt.t0, 0
    for d in pt.dt.tolist():
        if d == gnoc.PackedTrace.ESC:
            T, k = int(pt.abs_ps[k]), k + 1
        else:
            T += d
        out.append(T)
    assert k == pt.abs_ps.size
    assert np.array_equal(np.array(out, np.uint64), t)


def test_packed_wire_format_optional_arrays():
    """gnoc.PackedTrace keeps the length array only when lengths vary and the flag
    array only when a flag is set; the fields it keeps equal the trace's."""
    import numpy as np
    from graphite_amd import gnoc
    tr = gnoc.synthetic_trace(8, 8, 0.02, 300, seed=4).normalized()
    bits = tr.bits.copy()
    bits[::5] = 72
    flags = tr.flags.copy()
    flags[::7] |= gnoc.PKT_UNMODELED
    pt = gnoc.PackedTrace.of(gnoc.Trace(tr.inject_ps, tr.src, tr.dst, bits, flags))
    assert pt.bits is not None and pt.flags is not None
    assert np.array_equal(pt.bits, bits.astype(np.uint16)) and np.array_equal(pt.flags, flags.astype(np.uint8))
    assert np.array_equal(pt.src, tr.src.astype(np.uint16)) and np.array_equal(pt.dst, tr.dst.astype(np.uint16))
    assert pt.wire_bytes() == len(pt) * 9 + 8 * pt.abs_ps.size
    empty = gnoc.PackedTrace.of(gnoc.Trace(tr.inject_ps[:0], tr.src[:0], tr.dst[:0], tr.bits[:0], tr.flags[:0]))
    assert len(empty) == 0 and empty.abs_ps.size == 0 and empty.wire_bytes() == 0
