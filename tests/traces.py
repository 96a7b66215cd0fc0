"""Trace builders shared by the tests (small, seeded)."""
import numpy as np

from graphite_amd.gnoc import Trace, PKT_BROADCAST, PKT_UNMODELED


def random_trace(n, W, H, seed=0, max_cycle=200, burst0=0, self_frac=0.0, unmodeled_frac=0.0,
                 bits=576, bits_choices=None, ps_jitter=False, frequency_ghz=1.0, bcast_frac=0.0):
    """Random (time, id)-ordered trace; burst0 packets injected at t=0."""
    rng = np.random.default_rng(seed)
    N = W * H
    cyc = np.sort(rng.integers(0, max_cycle, n)).astype(np.uint64)
    cyc[:min(burst0, n)] = 0
    cyc = np.sort(cyc)
    one = int(np.ceil(1000.0 / frequency_ghz))
    t = cyc * np.uint64(one)
    if ps_jitter:
        t = np.sort(t + rng.integers(0, 700, n).astype(np.uint64))
    src = rng.integers(0, N, n).astype(np.uint32)
    dst = rng.integers(0, N, n).astype(np.uint32)
    if self_frac:
        m = rng.random(n) < self_frac
        dst[m] = src[m]
    flags = np.zeros(n, np.uint32)
    if unmodeled_frac:
        flags[rng.random(n) < unmodeled_frac] = PKT_UNMODELED
    if bcast_frac:
        flags[rng.random(n) < bcast_frac] |= PKT_BROADCAST
    if bits_choices is not None:
        b = rng.choice(np.asarray(bits_choices, np.uint32), n).astype(np.uint32)
    else:
        b = np.full(n, bits, np.uint32)
    return Trace(t, src, dst, b, flags)
