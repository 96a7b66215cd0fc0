"""Pipelined batches (gnoc_submit_async / gnoc_submit_commit / gnoc_fetch_final_ps):
batch k+1's upload and batch k's read-back run on copy streams beside the runs,
and every batch's results equal a one-batch-at-a-time run's (and the oracle's)."""
import numpy as np
import pytest
import torch

from graphite_amd import gnoc
from oracle import oracle

pytestmark = pytest.mark.gpu


def pinned(tr):
    def pin(x):
        t = torch.empty(x.shape[0], dtype={8: torch.int64, 4: torch.int32}[x.dtype.itemsize], pin_memory=True)
        v = t.numpy().view(x.dtype)
        v[:] = x
        return v
    return gnoc.Trace(pin(tr.inject_ps), pin(tr.src), pin(tr.dst), pin(tr.bits), pin(tr.flags))


def test_pipelined_batches_match_serial_runs():
    cfg = gnoc.EngineConfig(num_tiles=256)
    # different sizes and loads, so a stale buffer or a wrong swap shows up
    trs = [gnoc.synthetic_trace(16, 16, ld, ppt, seed=s) for ld, ppt, s in
           ((0.01, 400, 1), (0.03, 250, 2), (0.01, 400, 3), (0.05, 150, 4))]
    want = []
    eng = gnoc.Engine(cfg)
    for tr in trs:
        eng.submit(tr)
        eng.run()
        want.append(eng.results().final_ps.copy())
    eng.close()
    ptrs = [pinned(tr.normalized()) for tr in trs]
    outs = [torch.empty(len(tr), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64) for tr in trs]
    eng = gnoc.Engine(cfg)
    eng.submit(ptrs[0])
    for k in range(len(trs)):
        if k + 1 < len(trs):
            eng.submit_async(ptrs[k + 1])
        eng.run()
        eng.fetch_final_ps(outs[k])
        if k + 1 < len(trs):
            eng.submit_commit()
    eng.fetch_wait()
    last = eng.results()
    eng.close()
    for k in range(len(trs)):
        assert np.array_equal(outs[k], want[k]), f"batch {k}"
    assert np.array_equal(last.final_ps, want[-1])
    assert np.array_equal(outs[0], oracle.run(cfg, trs[0]).final_ps)


def test_pipeline_state_errors():
    cfg = gnoc.EngineConfig(num_tiles=16)
    tr = gnoc.synthetic_trace(4, 4, 0.02, 50, seed=5)
    eng = gnoc.Engine(cfg)
    with pytest.raises(gnoc.GnocError):
        eng.submit_commit()                       # nothing staged
    eng.submit(tr)
    with pytest.raises(gnoc.GnocError):
        eng.fetch_final_ps(np.empty(len(tr), np.uint64))   # no run yet
    eng.submit_async(tr)
    with pytest.raises(gnoc.GnocError):
        eng.submit_async(tr)                      # one staged batch at a time
    eng.submit_commit()
    eng.run()
    out = np.empty(len(tr), np.uint64)
    eng.fetch_final_ps(out)
    eng.fetch_wait()
    assert np.array_equal(out, eng.results().final_ps)
    eng.close()


def test_narrow_wire_format_matches_wide():
    """gnoc_submit_narrow / gnoc_submit_async_narrow (u16 ids and lengths, u8 flags,
    widened on the device) give the same results as the 24-B format, self-sends and
    unmodeled packets included; traces that do not fit are refused on the host."""
    from tests.traces import random_trace
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(5000, 8, 8, seed=17, max_cycle=3000, burst0=5, self_frac=0.05)
    tr.flags[::37] |= gnoc.PKT_UNMODELED
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    want = eng.results()
    nt = gnoc.NarrowTrace.of(tr)
    eng.submit_narrow(nt)
    eng.run()
    got = eng.results()
    for k in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_flit"):
        assert np.array_equal(getattr(got, k), getattr(want, k)), k
    eng.submit_async_narrow(nt)
    eng.submit_commit()
    eng.run()
    assert np.array_equal(eng.results().final_ps, want.final_ps)
    eng.close()
    big = gnoc.Trace(tr.inject_ps, tr.src, tr.dst, tr.bits.copy(), tr.flags)
    big.bits[0] = 1 << 16
    with pytest.raises(ValueError):
        gnoc.NarrowTrace.of(big)


@pytest.mark.parametrize("case", ["one_length", "mixed", "gaps"])
def test_packed_wire_format_matches_wide(case):
    """gnoc_submit_packed / gnoc_submit_async_packed (u16 inject-time differences with
    absolute-time escapes, decoded on the device by a segmented scan) give the same
    results as the 24-B format: one modeled length and no flags (6 B per packet),
    mixed lengths with unmodeled packets, and idle gaps longer than the u16
    difference (escapes in many decode blocks, including two in a row)."""
    from tests.traces import random_trace
    cfg = gnoc.EngineConfig(num_tiles=64)
    if case == "one_length":
        tr = gnoc.synthetic_trace(8, 8, 0.02, 800, seed=5)
    else:
        tr = random_trace(9000, 8, 8, seed=19, max_cycle=6000, burst0=5, self_frac=0.05)
        if case == "mixed":
            tr.flags[::41] |= gnoc.PKT_UNMODELED
        else:
            t = tr.inject_ps.astype(np.uint64)
            t[3000:] += np.uint64(70_000_000)      # one long idle gap
            t[5000:] += np.uint64(123_457)         # another one
            t[5001:] += np.uint64(65_535)          # and an escape right behind it
            tr = gnoc.Trace(t, tr.src, tr.dst, tr.bits, tr.flags)
    pt = gnoc.PackedTrace.of(tr)
    if case == "one_length":
        assert pt.bits is None and pt.flags is None and pt.wire_bytes() <= 6 * len(pt) + 8 * pt.abs_ps.size
    if case == "gaps":
        assert pt.abs_ps.size >= 3
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    want = eng.results()
    eng.submit_packed(pt)
    eng.run()
    got = eng.results()
    for k in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_flit"):
        assert np.array_equal(getattr(got, k), getattr(want, k)), k
    eng.submit_async_packed(pt)
    eng.submit_commit()
    eng.run()
    assert np.array_equal(eng.results().final_ps, want.final_ps)
    eng.close()


def test_pipelined_latency_readback_matches_final_ps():
    """gnoc_fetch_latency: the u32 latency (final_ps - inject_ps) read back on the
    copy stream, pipelined across batches of different sizes; the first call of an
    engine computes the array of the run before it, later runs write it in k_finalize."""
    cfg = gnoc.EngineConfig(num_tiles=256)
    trs = [gnoc.synthetic_trace(16, 16, ld, ppt, seed=s) for ld, ppt, s in
           ((0.01, 400, 1), (0.03, 250, 2), (0.05, 150, 4))]
    want = []
    eng = gnoc.Engine(cfg)
    for tr in trs:
        eng.submit(tr)
        eng.run()
        want.append((eng.results().final_ps - tr.inject_ps).astype(np.uint32))
    eng.close()
    ptrs = [pinned(tr.normalized()) for tr in trs]
    outs = [torch.empty(len(tr), dtype=torch.int32, pin_memory=True).numpy().view(np.uint32) for tr in trs]
    eng = gnoc.Engine(cfg)
    eng.submit(ptrs[0])
    for k in range(len(trs)):
        if k + 1 < len(trs):
            eng.submit_async(ptrs[k + 1])
        eng.run()
        eng.fetch_latency(outs[k])
        if k + 1 < len(trs):
            eng.submit_commit()
    eng.fetch_wait()
    eng.close()
    for k in range(len(trs)):
        assert np.array_equal(outs[k], want[k]), f"batch {k}"


def test_latency_readback_refuses_overflow():
    """A latency of 2^32 ps or more cannot be read back as u32: a burst of 130 K
    36-flit packets into one tile at cycle 0 (FIFO queues) queues the last one ~4.7 M
    cycles; gnoc_fetch_latency refuses, gnoc_fetch_final_ps still works."""
    n = 130000
    cfg = gnoc.EngineConfig(num_tiles=16, flit_width=16, analytical_enabled=False)
    rng = np.random.default_rng(3)
    src = rng.integers(1, 16, n).astype(np.uint32)
    tr = gnoc.Trace(np.zeros(n, np.uint64), src, np.zeros(n, np.uint32), np.full(n, 576, np.uint32),
                    np.zeros(n, np.uint32))
    eng = gnoc.Engine(cfg)
    eng.submit(pinned(tr))
    eng.run()
    fin = eng.results().final_ps
    assert int(fin.max()) >= 1 << 32
    out = torch.empty(n, dtype=torch.int32, pin_memory=True).numpy().view(np.uint32)
    with pytest.raises(gnoc.GnocError):
        eng.fetch_latency(out)
    f64 = torch.empty(n, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
    eng.fetch_final_ps(f64)
    eng.fetch_wait()
    assert np.array_equal(f64, fin)
    eng.close()


@pytest.mark.parametrize("n,esc_every", [(0, 0), (1, 0), (2047, 0), (2048, 1), (2049, 2048), (6145, 7), (4097, 2047)])
def test_packed_decode_block_edges(n, esc_every):
    """The delta decode's segmented scan at its block edges (2,048 packets per
    decode block): batch sizes around one and several blocks, escapes on every
    packet, at block boundaries and scattered; the decoded inject times (read back
    as final_ps - latency of a contention-free run, i.e. through the whole path)
    equal the 24-B upload's results."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    rng = np.random.default_rng(n + esc_every)
    gaps = rng.integers(0, 3, n).astype(np.uint64) * np.uint64(1000)
    if esc_every:
        gaps[::esc_every] += np.uint64(70_000)          # differences that need an escape
    t = np.cumsum(gaps, dtype=np.uint64) + np.uint64(5_000)
    src = rng.integers(0, 64, n).astype(np.uint32)
    dst = rng.integers(0, 64, n).astype(np.uint32)
    tr = gnoc.Trace(t, src, dst, np.full(n, 576, np.uint32), np.zeros(n, np.uint32))
    pt = gnoc.PackedTrace.of(tr)
    if esc_every == 1:
        assert pt.abs_ps.size == n - 1   # (the first packet is t0 itself)
    eng = gnoc.Engine(cfg)
    eng.submit(tr)
    eng.run()
    want = eng.results().final_ps.copy()
    eng.submit_packed(pt)
    eng.run()
    assert np.array_equal(eng.results().final_ps, want)
    eng.close()


def test_packed_escape_count_is_checked():
    """A delta-format batch whose 0xFFFF escapes do not match the absolute times it
    gives (n_abs) is refused by the submit's checks (synchronous and staged).  The
    decoder never reads past the n_abs given times (an escape beyond them decodes
    as 0, engine.hip pk_abs); k_pk_check's count mismatch is what refuses the batch."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    t = (np.arange(3000, dtype=np.uint64) * np.uint64(40_000))   # every difference escapes
    rng = np.random.default_rng(5)
    tr = gnoc.Trace(t, rng.integers(0, 64, 3000).astype(np.uint32), rng.integers(0, 64, 3000).astype(np.uint32),
                    np.full(3000, 576, np.uint32), np.zeros(3000, np.uint32))
    pt = gnoc.PackedTrace.of(tr)
    assert pt.abs_ps.size == 0   # 40,000 ps differences fit below 0xFFFF
    bad = gnoc.PackedTrace(pt.t0, pt.dt.copy(), np.array([7], np.uint64), pt.src, pt.dst, pt.bits, pt.bits_all, pt.flags)
    bad.dt[1000] = gnoc.PackedTrace.ESC
    bad.dt[1001] = gnoc.PackedTrace.ESC   # two escapes, one absolute time
    eng = gnoc.Engine(cfg)
    with pytest.raises(gnoc.GnocError, match="escapes"):
        eng.submit_packed(bad)
    eng.submit(tr)
    eng.run()
    eng.submit_async_packed(bad)
    with pytest.raises(gnoc.GnocError, match="escapes"):
        eng.submit_commit()
    eng.submit_packed(pt)          # a correct one still goes through
    eng.run()
    eng.close()


@pytest.mark.parametrize("nesc", [1, 700, 5000])
def test_packed_escapes_without_absolute_times_are_refused(nesc):
    """n_abs = 0 with escapes spread over many decode blocks (2,048
    packets each).  Every escape ordinal is past the (empty) absolute-time array:
    the decode stays in bounds and the submit is refused, synchronous and staged,
    and the engine takes the next good batch."""
    cfg = gnoc.EngineConfig(num_tiles=64)
    n = 20000
    rng = np.random.default_rng(nesc)
    t = np.sort(rng.integers(0, 40_000_000, n)).astype(np.uint64)
    tr = gnoc.Trace(t, rng.integers(0, 64, n).astype(np.uint32), rng.integers(0, 64, n).astype(np.uint32),
                    np.full(n, 576, np.uint32), np.zeros(n, np.uint32))
    pt = gnoc.PackedTrace.of(tr)
    dt = pt.dt.copy()
    dt[rng.choice(n, nesc, replace=False)] = gnoc.PackedTrace.ESC
    bad = gnoc.PackedTrace(pt.t0, dt, np.zeros(0, np.uint64), pt.src, pt.dst, pt.bits, pt.bits_all, pt.flags)
    eng = gnoc.Engine(cfg)
    with pytest.raises(gnoc.GnocError, match="escapes"):
        eng.submit_packed(bad)
    eng.submit_async_packed(bad)
    with pytest.raises(gnoc.GnocError, match="escapes"):
        eng.submit_commit()
    eng.submit_packed(pt)
    eng.run()
    np.testing.assert_array_equal(eng.results().final_ps, oracle.run(cfg, tr).final_ps)
    eng.close()
