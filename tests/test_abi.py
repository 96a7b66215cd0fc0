"""CPU-side checks of the C ABI library: it loads, exports every symbol the
header declares, and its host-only helpers behave (no GPU calls here)."""
import ctypes
import os
import re

import numpy as np

from graphite_amd import gnoc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "gnoc.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(gnoc_[a-z_]+)\s*\(", hdr)))


def test_exports_every_declared_symbol():
    lib = gnoc.load()
    decl = declared_symbols()
    assert len(decl) >= 12
    for s in decl:
        assert hasattr(lib, s), s
    assert set(decl) == set(gnoc.EXPORTED)


def test_abi_version_and_defaults():
    lib = gnoc.load()
    assert lib.gnoc_abi_version() == 4 == gnoc.ABI_VERSION
    # the summary layout of ABI 3 (include/gnoc.h): 112 bytes, the cumulative counters last
    assert ctypes.sizeof(gnoc.GnocSummary) == 112
    assert gnoc.GnocSummary.runs.offset == 96 and gnoc.GnocSummary.abi_pad2.offset == 108
    c = gnoc.GnocConfig()
    lib.gnoc_config_default(ctypes.byref(c), 1024)
    assert (c.num_tiles, c.flit_width, c.router_delay, c.link_delay) == (1024, 64, 1, 1)
    assert (c.contention_enabled, c.analytical_enabled, c.max_list_size) == (1, 1, 100)
    assert c.frequency_ghz == 1.0 and c.tile_width_mm == 1.0


def test_build_id_names_the_sources():
    """gnoc_build_id is the SHA-256 prefix build() computed over the device sources
    and flags (profiles/ record it; bench.py pairs a PMC profile with the build)."""
    import __graft_entry__ as ge
    lib = gnoc.load()
    bid = lib.gnoc_build_id().decode()
    assert re.fullmatch(r"[0-9a-f]{16}", bid), bid
    assert bid == ge.build_id(), "libgnoc.so is stale: rebuild (__graft_entry__.build())"


def test_create_rejects_invalid_config_without_gpu():
    lib = gnoc.load()
    h = ctypes.c_void_p()
    bad = [dict(num_tiles=10), dict(num_tiles=16, link_delay=2), dict(num_tiles=16, flit_width=0),
           dict(num_tiles=16, max_list_size=1), dict(num_tiles=16, queue_type=3)]
    for kw in bad:
        c = gnoc.EngineConfig(**kw).to_c()
        c.mesh_width = c.mesh_height = 0
        assert lib.gnoc_create(ctypes.byref(c), ctypes.byref(h)) < 0, kw


def _glibc_drand48_seq(seed, k):
    libc = ctypes.CDLL("libc.so.6")
    buf = ctypes.create_string_buffer(64)
    libc.srand48_r(ctypes.c_long(seed), buf)
    out = []
    d = ctypes.c_double()
    for _ in range(k):
        libc.drand48_r(buf, ctypes.byref(d))
        out.append(d.value)
    return out


def test_synthetic_trace_restates_reference_generator():
    W = H = 4
    N = 16
    load, ppt, seed = 0.2, 30, 77
    tr = gnoc.synthetic_trace(W, H, load, ppt, seed=seed)
    assert len(tr) == N * ppt
    assert np.all(np.diff(tr.inject_ps.astype(np.int64)) >= 0)
    assert np.all(tr.bits == (64 + 8) * 8)
    # uniform_random LCG schedule (synthetic_network.cc:247-301)
    sm = np.zeros((N, N), np.int64)
    sm[0, 0] = N // 2
    for i in range(N):
        if i:
            sm[i, 0] = sm[i - 1, 1]
        for j in range(1, N):
            sm[i, j] = (13 * sm[i, j - 1] + 5) % N
    for t in range(N):
        m = tr.src == t
        cyc = tr.inject_ps[m] // 1000
        # Bernoulli draws with glibc drand48_r seeded seed + tile (canSendPacket :230-233)
        draws = _glibc_drand48_seq(seed + t, int(cyc[-1]) + 1)
        expect = [c for c, r in enumerate(draws) if r < load][:ppt]
        assert list(cyc) == expect
        assert list(tr.dst[m]) == [sm[k % N, t] for k in range(ppt)]
