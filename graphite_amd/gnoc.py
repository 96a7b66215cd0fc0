"""ctypes binding of the C ABI in include/gnoc.h (libgnoc.so).

This is plumbing for tests and bench.py: the product is the HIP engine behind
the C ABI.  Loading fails loudly if the built library is missing -- there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GNOC_LIB", os.path.join(_HERE, "_build", "libgnoc.so"))
ABI_VERSION = 4   # include/gnoc.h GNOC_ABI_VERSION (4: the packed format, gnoc_fetch_latency)

GNOC_OK = 0
GNOC_EINVAL = -1
GNOC_ETRACE = -2
GNOC_EHIP = -3
GNOC_ESTATE = -4
GNOC_EUNSUPPORTED = -5
GNOC_ENOMEM = -6

PORT_SELF, PORT_LEFT, PORT_RIGHT, PORT_DOWN, PORT_UP, PORT_INJ = range(6)
QUEUE_HISTORY_TREE, QUEUE_BASIC, QUEUE_HISTORY_LIST = 0, 1, 2
# queue_model/basic/moving_avg_type (moving_average.h:175-189); NONE = moving_avg_enabled false
MOVING_AVG_NONE, MOVING_AVG_ARITHMETIC_MEAN, MOVING_AVG_GEOMETRIC_MEAN, MOVING_AVG_MEDIAN = 0, 1, 2, 3
PORTS_PER_TILE = 6
PKT_UNMODELED = 0x1
PKT_BROADCAST = 0x2     # receiver = NetPacket::BROADCAST, routed on the broadcast tree

# Every symbol include/gnoc.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "gnoc_config_default", "gnoc_create", "gnoc_submit", "gnoc_submit_device", "gnoc_run",
    "gnoc_get_packet_results", "gnoc_get_port_stats", "gnoc_get_summary", "gnoc_device_final_ps",
    "gnoc_last_error", "gnoc_destroy", "gnoc_trace_synthetic", "gnoc_abi_version",
    "gnoc_set_profiling", "gnoc_get_kernel_stats", "gnoc_trace_file_write", "gnoc_trace_file_read",
    "gnoc_trace_file_write_q", "gnoc_trace_file_read_q", "gnoc_trace_synthetic_pattern",
    "gnoc_shard_set_comm", "gnoc_shard_set_transport", "gnoc_run_sharded",
    "gnoc_shard", "gnoc_exchange_counts", "gnoc_run_begin", "gnoc_run_finish",
    "gnoc_create_sweep", "gnoc_sweep_layout", "gnoc_get_port_utilization", "gnoc_create_hop_counter",
    "gnoc_get_broadcast_results", "gnoc_get_broadcast_info", "gnoc_set_basic_moving_average",
    "gnoc_build_id", "gnoc_rccl_unique_id", "gnoc_rccl_comm_init", "gnoc_rccl_comm_destroy",
    "gnoc_submit_async", "gnoc_submit_commit", "gnoc_fetch_final_ps", "gnoc_fetch_latency", "gnoc_fetch_wait",
    "gnoc_submit_narrow", "gnoc_submit_async_narrow", "gnoc_submit_packed", "gnoc_submit_async_packed",
    "gnoc_pack_trace",
)


class GnocConfig(ctypes.Structure):
    _fields_ = [
        ("mesh_width", ctypes.c_int32),
        ("mesh_height", ctypes.c_int32),
        ("num_tiles", ctypes.c_int32),
        ("flit_width", ctypes.c_int32),
        ("router_delay", ctypes.c_uint64),
        ("link_delay", ctypes.c_uint64),
        ("frequency_ghz", ctypes.c_double),
        ("tile_width_mm", ctypes.c_double),
        ("contention_enabled", ctypes.c_int32),
        ("queue_type", ctypes.c_int32),
        ("analytical_enabled", ctypes.c_int32),
        ("max_list_size", ctypes.c_int32),
        ("broadcast_tree_enabled", ctypes.c_int32),
        ("device", ctypes.c_int32),
    ]


class GnocPoint(ctypes.Structure):
    _fields_ = [
        ("flit_width", ctypes.c_int32),
        ("router_delay", ctypes.c_uint64),
        ("link_delay", ctypes.c_uint64),
        ("tile_width_mm", ctypes.c_double),
    ]


class GnocPackets(ctypes.Structure):
    _fields_ = [
        ("inject_ps", ctypes.c_void_p),
        ("src", ctypes.c_void_p),
        ("dst", ctypes.c_void_p),
        ("bits", ctypes.c_void_p),
        ("flags", ctypes.c_void_p),
    ]


class GnocPacketsPacked(ctypes.Structure):
    _fields_ = [
        ("t0", ctypes.c_uint64),
        ("dt", ctypes.c_void_p),
        ("abs_ps", ctypes.c_void_p),
        ("n_abs", ctypes.c_uint64),
        ("src", ctypes.c_void_p),
        ("dst", ctypes.c_void_p),
        ("bits", ctypes.c_void_p),
        ("bits_all", ctypes.c_uint32),
        ("pad", ctypes.c_uint32),
        ("flags", ctypes.c_void_p),
    ]


class GnocPackInfo(ctypes.Structure):
    _fields_ = [("t0", ctypes.c_uint64), ("n_abs", ctypes.c_uint64), ("bits_all", ctypes.c_uint32),
                ("flags_any", ctypes.c_uint32)]


class GnocPacketsNarrow(ctypes.Structure):
    _fields_ = [
        ("inject_ps", ctypes.c_void_p),
        ("src", ctypes.c_void_p),
        ("dst", ctypes.c_void_p),
        ("bits", ctypes.c_void_p),
        ("flags", ctypes.c_void_p),
    ]


class GnocTraceQueue(ctypes.Structure):
    _fields_ = [("ma_type", ctypes.c_int32), ("ma_window", ctypes.c_uint32)]


class GnocSummary(ctypes.Structure):
    _fields_ = [
        ("packets", ctypes.c_uint64),
        ("routed_packets", ctypes.c_uint64),
        ("mesh_hops", ctypes.c_uint64),
        ("records", ctypes.c_uint64),
        ("mg1_uses", ctypes.c_uint64),
        ("levels", ctypes.c_uint32),
        ("engine_path", ctypes.c_uint32),
        ("last_run_ms", ctypes.c_double),
        ("retries", ctypes.c_uint32),
        ("fallbacks", ctypes.c_uint32),
        ("windows", ctypes.c_uint32),
        ("window_shift", ctypes.c_uint32),
        ("windows_y", ctypes.c_uint32),
        ("chain_protocol", ctypes.c_uint32),
        ("window_ps_x", ctypes.c_uint64),
        ("window_ps_y", ctypes.c_uint64),
        ("runs", ctypes.c_uint32),
        ("retries_total", ctypes.c_uint32),
        ("fallbacks_total", ctypes.c_uint32),
        ("abi_pad2", ctypes.c_uint32),
    ]


_lib = None


def load() -> ctypes.CDLL:
    """Load libgnoc.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback exists)")
    # torch first, so libgnoc.so binds the HIP runtime torch loaded (one runtime per
    # process: a second one finds no devices)
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.gnoc_config_default.argtypes = [ctypes.POINTER(GnocConfig), ctypes.c_int32]
    lib.gnoc_config_default.restype = None
    lib.gnoc_create.argtypes = [ctypes.POINTER(GnocConfig), ctypes.POINTER(vp)]
    lib.gnoc_submit.argtypes = [vp, ctypes.POINTER(GnocPackets), sz]
    lib.gnoc_submit_device.argtypes = [vp, ctypes.POINTER(GnocPackets), sz]
    lib.gnoc_run.argtypes = [vp]
    lib.gnoc_get_packet_results.argtypes = [vp, vp, vp, vp, sz]
    lib.gnoc_get_port_stats.argtypes = [vp, vp, vp, vp, sz]
    lib.gnoc_get_summary.argtypes = [vp, ctypes.POINTER(GnocSummary)]
    lib.gnoc_get_port_utilization.argtypes = [vp, vp, vp, sz]
    lib.gnoc_device_final_ps.argtypes = [vp, ctypes.POINTER(vp)]
    lib.gnoc_last_error.argtypes = [vp]
    lib.gnoc_last_error.restype = ctypes.c_char_p
    lib.gnoc_destroy.argtypes = [vp]
    lib.gnoc_destroy.restype = None
    lib.gnoc_trace_synthetic.argtypes = [
        ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_uint64, ctypes.c_double, ctypes.c_int32, vp, vp, vp, vp, sz, ctypes.POINTER(sz)]
    lib.gnoc_trace_synthetic_pattern.argtypes = [
        ctypes.c_int32,
        ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_uint64, ctypes.c_uint32,
        ctypes.c_uint64, ctypes.c_double, ctypes.c_int32, vp, vp, vp, vp, sz, ctypes.POINTER(sz)]
    lib.gnoc_abi_version.argtypes = []
    # the summary layout (runs, retries_total, fallbacks_total, chain_protocol) is ABI 3-4's:
    # an older library would leave the rerun totals the bench checks at zero
    if lib.gnoc_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{LIB_PATH}: ABI {lib.gnoc_abi_version()}, this module speaks {ABI_VERSION}")
    if hasattr(lib, "gnoc_build_id"):
        lib.gnoc_build_id.argtypes = []
        lib.gnoc_build_id.restype = ctypes.c_char_p
    lib.gnoc_trace_file_write.argtypes = [ctypes.c_char_p, ctypes.POINTER(GnocConfig), ctypes.POINTER(GnocPackets), sz]
    lib.gnoc_trace_file_write_q.argtypes = [ctypes.c_char_p, ctypes.POINTER(GnocConfig), ctypes.POINTER(GnocTraceQueue),
                                            ctypes.POINTER(GnocPackets), sz]
    lib.gnoc_trace_file_read_q.argtypes = [ctypes.c_char_p, ctypes.POINTER(GnocConfig), ctypes.POINTER(GnocTraceQueue),
                                           vp, vp, vp, vp, vp, sz, ctypes.POINTER(sz)]
    lib.gnoc_trace_file_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(GnocConfig), vp, vp, vp, vp, vp, sz,
                                         ctypes.POINTER(sz)]
    lib.gnoc_set_profiling.argtypes = [vp, ctypes.c_int]
    lib.gnoc_get_kernel_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_uint32), sz, ctypes.POINTER(sz)]
    lib.gnoc_create_sweep.argtypes = [ctypes.POINTER(GnocConfig), ctypes.POINTER(GnocPoint), ctypes.c_int32,
                                      ctypes.POINTER(vp)]
    lib.gnoc_sweep_layout.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    lib.gnoc_create_hop_counter.argtypes = [ctypes.POINTER(GnocConfig), ctypes.POINTER(vp)]
    lib.gnoc_get_broadcast_results.argtypes = [vp, vp, vp, vp, sz]
    lib.gnoc_get_broadcast_info.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]
    lib.gnoc_shard.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
    lib.gnoc_exchange_counts.argtypes = [vp, vp, vp, sz]
    lib.gnoc_run_begin.argtypes = [vp, vp]
    lib.gnoc_run_finish.argtypes = [vp, vp]
    lib.gnoc_set_basic_moving_average.argtypes = [vp, ctypes.c_int32, ctypes.c_uint32]
    if hasattr(lib, "gnoc_submit_narrow"):
        lib.gnoc_submit_narrow.argtypes = [vp, ctypes.POINTER(GnocPacketsNarrow), sz]
        lib.gnoc_submit_async_narrow.argtypes = [vp, ctypes.POINTER(GnocPacketsNarrow), sz]
    if hasattr(lib, "gnoc_submit_packed"):
        lib.gnoc_submit_packed.argtypes = [vp, ctypes.POINTER(GnocPacketsPacked), sz]
        lib.gnoc_submit_async_packed.argtypes = [vp, ctypes.POINTER(GnocPacketsPacked), sz]
    lib.gnoc_pack_trace.argtypes = [ctypes.POINTER(GnocPackets), sz, vp, vp, vp, vp, vp, vp, sz,
                                    ctypes.POINTER(GnocPackInfo)]
    if hasattr(lib, "gnoc_submit_async"):
        lib.gnoc_submit_async.argtypes = [vp, ctypes.POINTER(GnocPackets), sz]
        lib.gnoc_submit_commit.argtypes = [vp]
        lib.gnoc_fetch_final_ps.argtypes = [vp, vp, sz]
        lib.gnoc_fetch_latency.argtypes = [vp, vp, sz]
        lib.gnoc_fetch_wait.argtypes = [vp]
    lib.gnoc_shard_set_comm.argtypes = [vp, vp]
    lib.gnoc_run_sharded.argtypes = [vp]
    if hasattr(lib, "gnoc_rccl_unique_id"):
        lib.gnoc_rccl_unique_id.argtypes = [vp]
        lib.gnoc_rccl_comm_init.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, ctypes.POINTER(vp)]
        lib.gnoc_rccl_comm_destroy.argtypes = [vp]
    _lib = lib
    return lib


class GnocError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gnoc error {code}: {msg}")
        self.code = code


@dataclass
class EngineConfig:
    """The carbon_sim.cfg keys the emesh_hop_by_hop path reads."""
    num_tiles: int = 64                     # general/total_cores
    mesh_width: int = 0                     # derived: floor(sqrt(N))
    mesh_height: int = 0                    # derived: ceil(N / W)
    flit_width: int = 64                    # network/emesh_hop_by_hop/flit_width
    router_delay: int = 1                   # network/emesh_hop_by_hop/router/delay
    link_delay: int = 1                     # network/emesh_hop_by_hop/link/delay
    frequency_ghz: float = 1.0              # network DVFS domain
    tile_width_mm: float = 1.0              # general/tile_width
    contention_enabled: bool = True         # network/emesh_hop_by_hop/queue_model/enabled
    queue_type: int = 0                     # QUEUE_HISTORY_TREE / QUEUE_BASIC / QUEUE_HISTORY_LIST
    analytical_enabled: bool = True         # queue_model/history_tree/analytical_model_enabled
    max_list_size: int = 100                # queue_model/history_tree/max_list_size
    broadcast_tree_enabled: bool = True
    device: int = 0
    # queue_model/history_list/interleaving_enabled: no effect on in-order requests
    # (include/gnoc.h); kept so the oracle can restate the list with it on or off
    interleaving_enabled: bool = True
    # queue_model/basic/moving_avg_{enabled,type,window_size} (queue_model_basic.cc:7-30):
    # MOVING_AVG_* (NONE = disabled) and the window; only with queue_type QUEUE_BASIC
    # (set through gnoc_set_basic_moving_average, not part of gnoc_config)
    moving_avg_type: int = 0
    moving_avg_window: int = 64

    @property
    def width(self) -> int:
        import math
        return self.mesh_width or int(math.floor(math.sqrt(self.num_tiles)))

    @property
    def height(self) -> int:
        import math
        return self.mesh_height or int(math.ceil(self.num_tiles / self.width))

    def to_c(self) -> GnocConfig:
        c = GnocConfig()
        for f in GnocConfig._fields_:   # interleaving_enabled is not an engine key
            v = getattr(self, f[0])
            setattr(c, f[0], int(v) if not isinstance(v, float) else v)
        return c


@dataclass
class Trace:
    inject_ps: np.ndarray
    src: np.ndarray
    dst: np.ndarray
    bits: np.ndarray
    flags: Optional[np.ndarray] = None

    def __len__(self) -> int:
        return int(self.inject_ps.shape[0])

    def normalized(self) -> "Trace":
        f = self.flags if self.flags is not None else np.zeros(len(self), np.uint32)
        return Trace(np.ascontiguousarray(self.inject_ps, np.uint64), np.ascontiguousarray(self.src, np.uint32),
                     np.ascontiguousarray(self.dst, np.uint32), np.ascontiguousarray(self.bits, np.uint32),
                     np.ascontiguousarray(f, np.uint32))


@dataclass
class NarrowTrace:
    """A trace in the narrow wire format (gnoc_packets_narrow): u16 tile ids and
    modeled lengths, u8 flags -- 15 bytes per packet over PCIe instead of 24."""
    inject_ps: np.ndarray
    src: np.ndarray
    dst: np.ndarray
    bits: np.ndarray
    flags: np.ndarray

    def __len__(self) -> int:
        return int(self.inject_ps.shape[0])

    @staticmethod
    def of(tr: "Trace", alloc=np.empty) -> "NarrowTrace":
        """Narrow a trace (ValueError if a tile id, length or flag does not fit);
        alloc(shape, dtype) places the arrays (e.g. in page-locked memory)."""
        tr = tr.normalized()
        n = len(tr)
        for name, a, lim in (("src", tr.src, 1 << 16), ("dst", tr.dst, 1 << 16), ("bits", tr.bits, 1 << 16),
                             ("flags", tr.flags, 1 << 8)):
            if n and int(a.max()) >= lim:
                raise ValueError(f"{name} does not fit the narrow wire format")
        out = []
        for a, dt in ((tr.inject_ps, np.uint64), (tr.src, np.uint16), (tr.dst, np.uint16), (tr.bits, np.uint16),
                      (tr.flags, np.uint8)):
            b = alloc((n,), dt)
            b[:] = a
            out.append(b)
        return NarrowTrace(*out)

    def packets(self) -> GnocPacketsNarrow:
        return GnocPacketsNarrow(self.inject_ps.ctypes.data, self.src.ctypes.data, self.dst.ctypes.data,
                                 self.bits.ctypes.data, self.flags.ctypes.data)


@dataclass
class PackedTrace:
    """A trace in the delta wire format (gnoc_packets_packed): u16 inject-time
    differences (0xFFFF = the next absolute time in abs_ps), u16 tile ids, and the
    modeled lengths / flags only where they vary -- 6 bytes per packet for a batch of
    one length without flags."""
    t0: int
    dt: np.ndarray
    abs_ps: np.ndarray
    src: np.ndarray
    dst: np.ndarray
    bits: object          # np.ndarray, or None (every packet has bits_all)
    bits_all: int
    flags: object         # np.ndarray, or None (all zero)

    ESC = 0xFFFF

    def __len__(self) -> int:
        return int(self.dt.shape[0])

    @staticmethod
    def of(tr: "Trace", alloc=np.empty) -> "PackedTrace":
        """Pack a trace (ValueError if a tile id, length or flag does not fit the
        narrow fields) with the library's encoder (gnoc_pack_trace, the host's
        cores); alloc(shape, dtype) places the arrays (e.g. page-locked)."""
        tr = tr.normalized()
        lib = load()
        n = len(tr)
        dt, src, dst = alloc((n,), np.uint16), alloc((n,), np.uint16), alloc((n,), np.uint16)
        bits, flags = np.empty(n, np.uint16), np.empty(n, np.uint8)
        cap = n // 64 + 64
        for _ in range(2):
            absv = alloc((cap,), np.uint64)
            info = GnocPackInfo()
            pk = GnocPackets(tr.inject_ps.ctypes.data, tr.src.ctypes.data, tr.dst.ctypes.data, tr.bits.ctypes.data,
                             tr.flags.ctypes.data)
            rc = lib.gnoc_pack_trace(ctypes.byref(pk), n, dt.ctypes.data, src.ctypes.data, dst.ctypes.data,
                                     bits.ctypes.data, flags.ctypes.data, absv.ctypes.data, cap, ctypes.byref(info))
            if rc == 0 or info.n_abs <= cap:
                break
            cap = int(info.n_abs)
        if rc:
            raise ValueError("the trace does not fit the packed wire format")
        one_len = info.bits_all != 0xFFFFFFFF
        if one_len:
            bits = None
        else:
            b = alloc((n,), np.uint16)
            b[:] = bits
            bits = b
        if info.flags_any:
            f = alloc((n,), np.uint8)
            f[:] = flags
            flags = f
        else:
            flags = None
        na = int(info.n_abs)
        if na < cap:
            a2 = alloc((na,), np.uint64)
            a2[:] = absv[:na]
            absv = a2
        return PackedTrace(int(info.t0), dt, absv, src, dst, bits, int(info.bits_all) if one_len and n else 0, flags)

    @staticmethod
    def of_numpy(tr: "Trace", alloc=np.empty) -> "PackedTrace":
        """The same encoding in numpy (the reference the library's encoder is tested against)."""
        tr = tr.normalized()
        n = len(tr)
        for name, a, lim in (("src", tr.src, 1 << 16), ("dst", tr.dst, 1 << 16), ("bits", tr.bits, 1 << 16),
                             ("flags", tr.flags, 1 << 8)):
            if n and int(a.max()) >= lim:
                raise ValueError(f"{name} does not fit the packed wire format")
        t = tr.inject_ps.astype(np.uint64)
        t0 = int(t[0]) if n else 0
        d = np.diff(t, prepend=np.uint64(t0)) if n else np.zeros(0, np.uint64)
        esc = d >= PackedTrace.ESC

        def put(a, dt):
            b = alloc((a.shape[0],), dt)
            b[:] = a
            return b
        dt16 = put(np.where(esc, PackedTrace.ESC, d).astype(np.uint16), np.uint16)
        absv = put(t[esc], np.uint64)
        one_len = n == 0 or bool((tr.bits == tr.bits[0]).all())
        bits = None if one_len else put(tr.bits.astype(np.uint16), np.uint16)
        flags = None if n == 0 or not tr.flags.any() else put(tr.flags.astype(np.uint8), np.uint8)
        return PackedTrace(t0, dt16, absv, put(tr.src.astype(np.uint16), np.uint16), put(tr.dst.astype(np.uint16), np.uint16),
                           bits, int(tr.bits[0]) if n and one_len else 0, flags)

    def wire_bytes(self) -> int:
        return int(self.dt.nbytes + self.abs_ps.nbytes + self.src.nbytes + self.dst.nbytes +
                   (self.bits.nbytes if self.bits is not None else 0) + (self.flags.nbytes if self.flags is not None else 0))

    def packets(self) -> GnocPacketsPacked:
        return GnocPacketsPacked(self.t0, self.dt.ctypes.data, self.abs_ps.ctypes.data if self.abs_ps.size else None,
                                 int(self.abs_ps.size), self.src.ctypes.data, self.dst.ctypes.data,
                                 self.bits.ctypes.data if self.bits is not None else None, self.bits_all, 0,
                                 self.flags.ctypes.data if self.flags is not None else None)


# synthetic_network.cc NetworkTrafficType (:16-24), include/gnoc.h GNOC_TRAFFIC_*
TRAFFIC_PATTERNS = ("uniform_random", "bit_complement", "shuffle", "transpose", "tornado", "nearest_neighbor")


def synthetic_trace(width: int, height: int, offered_load: float, packets_per_tile: int, seed: int = 1,
                    payload_bytes: int = 8, frequency_ghz: float = 1.0, hotspot_fraction: float = 0.0,
                    num_hotspots: int = 16, pattern: str = "uniform_random") -> Trace:
    lib = load()
    pat = TRAFFIC_PATTERNS.index(pattern)
    n = ctypes.c_size_t(0)
    rc = lib.gnoc_trace_synthetic_pattern(pat, width, height, frequency_ghz, offered_load, packets_per_tile,
                                          payload_bytes, seed, hotspot_fraction, num_hotspots, None, None, None, None,
                                          0, ctypes.byref(n))
    if rc:
        raise GnocError(rc, "trace size query failed")
    N = n.value
    t = Trace(np.empty(N, np.uint64), np.empty(N, np.uint32), np.empty(N, np.uint32), np.empty(N, np.uint32),
              np.zeros(N, np.uint32))
    rc = lib.gnoc_trace_synthetic_pattern(pat, width, height, frequency_ghz, offered_load, packets_per_tile,
                                          payload_bytes, seed, hotspot_fraction, num_hotspots, t.inject_ps.ctypes.data,
                                          t.src.ctypes.data, t.dst.ctypes.data, t.bits.ctypes.data, N, ctypes.byref(n))
    if rc:
        raise GnocError(rc, f"synthetic trace generation failed ({pattern} on {width}x{height})")
    return t


def write_trace_file(path: str, cfg: "EngineConfig", tr: Trace) -> None:
    """The on-disk trace format of include/gnoc.h (gnoc_trace_header v2 + SoA),
    with the basic queue's moving-average settings of cfg."""
    lib = load()
    tr = tr.normalized()
    c = cfg.to_c()
    q = GnocTraceQueue(int(cfg.moving_avg_type), int(cfg.moving_avg_window if cfg.moving_avg_type else 1))
    pk = GnocPackets(tr.inject_ps.ctypes.data, tr.src.ctypes.data, tr.dst.ctypes.data, tr.bits.ctypes.data,
                     tr.flags.ctypes.data)
    rc = lib.gnoc_trace_file_write_q(path.encode(), ctypes.byref(c), ctypes.byref(q), ctypes.byref(pk), len(tr))
    if rc:
        raise GnocError(rc, f"cannot write trace {path}")


def read_trace_file(path: str):
    """-> (EngineConfig, Trace); a version-1 file reads with no moving average."""
    lib = load()
    c = GnocConfig()
    q = GnocTraceQueue()
    n = ctypes.c_size_t(0)
    rc = lib.gnoc_trace_file_read_q(path.encode(), ctypes.byref(c), ctypes.byref(q), None, None, None, None, None, 0,
                                    ctypes.byref(n))
    if rc:
        raise GnocError(rc, f"cannot read trace {path}")
    N = n.value
    t = Trace(np.empty(N, np.uint64), np.empty(N, np.uint32), np.empty(N, np.uint32), np.empty(N, np.uint32),
              np.empty(N, np.uint32))
    rc = lib.gnoc_trace_file_read(path.encode(), None, t.inject_ps.ctypes.data, t.src.ctypes.data, t.dst.ctypes.data,
                                  t.bits.ctypes.data, t.flags.ctypes.data, N, ctypes.byref(n))
    if rc:
        raise GnocError(rc, f"corrupt trace {path}")
    cfg = EngineConfig(**{f[0]: getattr(c, f[0]) for f in GnocConfig._fields_})
    for k in ("contention_enabled", "analytical_enabled", "broadcast_tree_enabled"):
        setattr(cfg, k, bool(getattr(cfg, k)))
    cfg.moving_avg_type = q.ma_type
    if q.ma_type:
        cfg.moving_avg_window = q.ma_window
    return cfg, t


@dataclass
class Results:
    final_ps: np.ndarray
    zero_load_ps: np.ndarray
    contention_ps: np.ndarray
    port_sum_delay: np.ndarray
    port_count: np.ndarray
    port_mg1: np.ndarray
    summary: dict = field(default_factory=dict)
    port_flit: Optional[np.ndarray] = None   # QueueModel _total_utilized_cycles (gnoc_get_port_utilization)
    port_last: Optional[np.ndarray] = None   # QueueModel _last_request_time
    # broadcast receipts [broadcast in trace order, receiving tile] (gnoc_get_broadcast_results)
    bcast_final_ps: Optional[np.ndarray] = None
    bcast_zero_load_ps: Optional[np.ndarray] = None
    bcast_contention_ps: Optional[np.ndarray] = None


def expand_broadcasts(tr: Trace, num_tiles: int) -> Trace:
    """What Network::netSend does with a broadcast when the model has no
    broadcast tree (network.cc:186-195): one unicast per tile, in tile order,
    at the broadcast's place in the trace.  (The reference also sends to the
    two system tiles; those hops are direct and time nothing, network_model.cc:431-436.)"""
    tr = tr.normalized()
    bc = (tr.flags & PKT_BROADCAST) != 0
    reps = np.where(bc, num_tiles, 1)
    idx = np.repeat(np.arange(len(tr)), reps)
    dst = tr.dst[idx].copy()
    first = np.cumsum(reps) - reps
    for i in np.nonzero(bc)[0]:
        dst[first[i]:first[i] + num_tiles] = np.arange(num_tiles, dtype=np.uint32)
    return Trace(tr.inject_ps[idx], tr.src[idx], dst, tr.bits[idx], tr.flags[idx] & ~np.uint32(PKT_BROADCAST))


class Engine:
    """One engine handle per GPU (gnoc_create; model="emesh_hop_counter":
    gnoc_create_hop_counter)."""

    def __init__(self, cfg: EngineConfig, model: str = "emesh_hop_by_hop"):
        self.lib = load()
        self.cfg = cfg
        self._h = ctypes.c_void_p()
        c = cfg.to_c()
        create = self.lib.gnoc_create_hop_counter if model == "emesh_hop_counter" else self.lib.gnoc_create
        rc = create(ctypes.byref(c), ctypes.byref(self._h))
        if model == "emesh_hop_counter":
            import math
            w = int(math.floor(math.sqrt(cfg.num_tiles)))
            from dataclasses import replace
            self.cfg = replace(cfg, mesh_width=w, mesh_height=int(math.ceil(cfg.num_tiles / w)))
        if rc:
            raise GnocError(rc, "gnoc_create rejected the configuration")
        if cfg.moving_avg_type and model != "emesh_hop_counter":
            self._check(self.lib.gnoc_set_basic_moving_average(self._h, cfg.moving_avg_type, cfg.moving_avg_window))
        self._n = 0
        self._keep = None

    def _check(self, rc: int) -> None:
        if rc:
            raise GnocError(rc, self.lib.gnoc_last_error(self._h).decode())

    def close(self) -> None:
        if self._h:
            self.lib.gnoc_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def submit(self, tr: Trace) -> None:
        tr = tr.normalized()
        pk = GnocPackets(tr.inject_ps.ctypes.data, tr.src.ctypes.data, tr.dst.ctypes.data, tr.bits.ctypes.data,
                         tr.flags.ctypes.data)
        self._check(self.lib.gnoc_submit(self._h, ctypes.byref(pk), len(tr)))
        self._n = len(tr)

    def submit_device(self, inject_ps: int, src: int, dst: int, bits: int, flags: int, n: int, keep=None) -> None:
        """Arrays already resident in HBM (device pointers, e.g. torch tensor data_ptr())."""
        pk = GnocPackets(inject_ps, src, dst, bits, flags)
        self._check(self.lib.gnoc_submit_device(self._h, ctypes.byref(pk), n))
        self._n = n
        self._keep = keep

    def run(self) -> None:
        self._check(self.lib.gnoc_run(self._h))

    # pipelined batches (gnoc_submit_async / _commit, gnoc_fetch_final_ps / _wait)
    def submit_async(self, tr: "Trace") -> None:
        """Start uploading the next batch (page-locked arrays overlap with the run
        in flight); it becomes current at submit_commit()."""
        tr = tr.normalized()
        pk = GnocPackets(tr.inject_ps.ctypes.data, tr.src.ctypes.data, tr.dst.ctypes.data, tr.bits.ctypes.data,
                         tr.flags.ctypes.data)
        self._check(self.lib.gnoc_submit_async(self._h, ctypes.byref(pk), len(tr)))
        self._staged = (tr, len(tr))

    def submit_narrow(self, nt: "NarrowTrace") -> None:
        """gnoc_submit_narrow: the 15-byte-per-packet wire format (widened on the device)."""
        self._check(self.lib.gnoc_submit_narrow(self._h, ctypes.byref(nt.packets()), len(nt)))
        self._n = len(nt)

    def submit_async_narrow(self, nt: "NarrowTrace") -> None:
        self._check(self.lib.gnoc_submit_async_narrow(self._h, ctypes.byref(nt.packets()), len(nt)))
        self._staged = (nt, len(nt))

    def submit_packed(self, pt: "PackedTrace") -> None:
        """gnoc_submit_packed: the delta wire format (decoded on the device)."""
        self._check(self.lib.gnoc_submit_packed(self._h, ctypes.byref(pt.packets()), len(pt)))
        self._n = len(pt)

    def submit_async_packed(self, pt: "PackedTrace") -> None:
        self._check(self.lib.gnoc_submit_async_packed(self._h, ctypes.byref(pt.packets()), len(pt)))
        self._staged = (pt, len(pt))

    def submit_commit(self) -> None:
        self._check(self.lib.gnoc_submit_commit(self._h))
        self._n = self._staged[1]
        self._staged = None

    def fetch_final_ps(self, out: np.ndarray) -> None:
        """Start copying the last run's final_ps into `out` (page-locked uint64 of
        the batch size); complete after fetch_wait()."""
        assert out.dtype.itemsize == 8 and out.shape[0] == self._n and out.flags["C_CONTIGUOUS"]
        self._check(self.lib.gnoc_fetch_final_ps(self._h, out.ctypes.data, self._n))

    def fetch_latency(self, out: np.ndarray) -> None:
        """Start copying the last run's per-packet latency (final_ps - inject_ps, u32
        ps) into `out` (page-locked uint32 of the batch size): half the bytes of
        final_ps; complete after fetch_wait()."""
        assert out.dtype.itemsize == 4 and out.shape[0] == self._n and out.flags["C_CONTIGUOUS"]
        self._check(self.lib.gnoc_fetch_latency(self._h, out.ctypes.data, self._n))

    def fetch_wait(self) -> None:
        self._check(self.lib.gnoc_fetch_wait(self._h))

    def summary(self) -> dict:
        s = GnocSummary()
        self._check(self.lib.gnoc_get_summary(self._h, ctypes.byref(s)))
        return {f[0]: getattr(s, f[0]) for f in GnocSummary._fields_ }

    def final_ps_into(self, out: np.ndarray) -> None:
        """final_ps only, into a caller's (e.g. pinned) uint64 array of the batch size."""
        assert out.dtype.itemsize == 8 and out.shape[0] == self._n and out.flags["C_CONTIGUOUS"]
        self._check(self.lib.gnoc_get_packet_results(self._h, out.ctypes.data, None, None, self._n))

    def results(self) -> Results:
        n = self._n
        fin, zl, ct = (np.empty(n, np.uint64) for _ in range(3))
        self._check(self.lib.gnoc_get_packet_results(self._h, fin.ctypes.data, zl.ctypes.data, ct.ctypes.data, n))
        npt = self.cfg.width * self.cfg.height * PORTS_PER_TILE
        ps, pc, pm = (np.empty(npt, np.uint64) for _ in range(3))
        self._check(self.lib.gnoc_get_port_stats(self._h, ps.ctypes.data, pc.ctypes.data, pm.ctypes.data, npt))
        pf, pl = np.empty(npt, np.uint64), np.empty(npt, np.uint64)
        self._check(self.lib.gnoc_get_port_utilization(self._h, pf.ctypes.data, pl.ctypes.data, npt))
        nb, _ = self.broadcast_info()
        N = self.cfg.width * self.cfg.height
        bf, bz, bt = (np.empty((nb, N), np.uint64) for _ in range(3))
        if nb:
            self._check(self.lib.gnoc_get_broadcast_results(self._h, bf.ctypes.data, bz.ctypes.data, bt.ctypes.data,
                                                            nb * N))
        return Results(fin, zl, ct, ps, pc, pm, self.summary(), pf, pl, bf, bz, bt)

    def broadcast_info(self):
        """-> (broadcast packets submitted, passes the last run took)"""
        nb, passes = ctypes.c_uint64(), ctypes.c_uint32()
        self._check(self.lib.gnoc_get_broadcast_info(self._h, ctypes.byref(nb), ctypes.byref(passes)))
        return int(nb.value), int(passes.value)

    def set_profiling(self, on: bool) -> None:
        self._check(self.lib.gnoc_set_profiling(self._h, int(on)))

    def kernel_stats(self) -> dict:
        """{kernel class: (total device ms over the last run, launches)}"""
        cap = 32
        names = (ctypes.c_char_p * cap)()
        ms = (ctypes.c_double * cap)()
        ln = (ctypes.c_uint32 * cap)()
        cnt = ctypes.c_size_t()
        self._check(self.lib.gnoc_get_kernel_stats(self._h, names, ms, ln, cap, ctypes.byref(cnt)))
        return {names[i].decode(): (ms[i], ln[i]) for i in range(min(cnt.value, cap))}

    def device_final_ps(self) -> int:
        p = ctypes.c_void_p()
        self._check(self.lib.gnoc_device_final_ps(self._h, ctypes.byref(p)))
        return int(p.value)


def band(b: int, n: int, dim: int) -> range:
    """Rows (or columns) of band b of n: [b*dim/n, (b+1)*dim/n) -- gnoc_shard's split."""
    return range(b * dim // n, (b + 1) * dim // n)


def turn_counts(tr: Trace, width: int, height: int, nranks: int) -> np.ndarray:
    """[r, d]: routed packets whose turn record moves from row band r (source row)
    to column band d (destination column): what gnoc_exchange_counts is built from."""
    tr = tr.normalized()
    routed = (tr.src != tr.dst) & ((tr.flags & PKT_UNMODELED) == 0)
    sy = (tr.src[routed] // width).astype(np.int64)
    dx = (tr.dst[routed] % width).astype(np.int64)
    rb = np.empty(height, np.int64)
    cb = np.empty(width, np.int64)
    for b in range(nranks):
        rb[band(b, nranks, height).start:band(b, nranks, height).stop] = b
        cb[band(b, nranks, width).start:band(b, nranks, width).stop] = b
    m = np.zeros((nranks, nranks), np.int64)
    np.add.at(m, (rb[sy], cb[dx]), 1)
    return m


def exchange_units(send, recv, send_units, recv_units, group=None) -> None:
    """The turn-record all-to-all: send[: sum(send_units)] (16-byte units, peers in
    rank order) -> recv[: sum(recv_units)].  "nccl" (RCCL over xGMI): device to
    device on torch's current stream, then synchronised so the engine's stream can
    read it; "gloo": staged through host memory (CPU tensors pass straight through)."""
    import torch
    import torch.distributed as dist
    s = send[:sum(send_units)]
    r = recv[:sum(recv_units)]
    if dist.get_backend(group) == "nccl":
        dist.all_to_all_single(r, s, output_split_sizes=recv_units, input_split_sizes=send_units, group=group)
        torch.cuda.current_stream().synchronize()
        return
    rh = r if r.device.type == "cpu" else torch.empty(r.shape, dtype=r.dtype)
    dist.all_to_all_single(rh, s.cpu(), output_split_sizes=recv_units, input_split_sizes=send_units, group=group)
    if rh is not r:
        r.copy_(rh)
        torch.cuda.synchronize()


class ShardedEngine(Engine):
    """One rank's share of a mesh sharded over torch.distributed ranks (gnoc_shard):
    row band for the X phase, column band for the Y phase, one all-to-all of the
    turn records in between.  With the "nccl" backend (RCCL over xGMI) the
    exchange runs device to device; with "gloo" it is staged through host memory
    (multi-process tests on one GPU or on CPU hosts)."""

    def __init__(self, cfg: EngineConfig, rank: int, nranks: int, group=None):
        super().__init__(cfg)
        self.rank, self.nranks, self.group = rank, nranks, group
        self._check(self.lib.gnoc_shard(self._h, rank, nranks))
        self._send = self._recv = None

    def submit(self, tr: Trace) -> None:
        import torch
        super().submit(tr)
        s = np.zeros(self.nranks, np.uint64)
        r = np.zeros(self.nranks, np.uint64)
        self._check(self.lib.gnoc_exchange_counts(self._h, s.ctypes.data, r.ctypes.data, self.nranks))
        self.send_units, self.recv_units = [int(v) for v in s], [int(v) for v in r]
        dev = torch.device("cuda", self.cfg.device)
        # 16-byte units as int32 x 4 (one Rec per unit)
        self._send = torch.empty((max(1, sum(self.send_units)), 4), dtype=torch.int32, device=dev)
        self._recv = torch.empty((max(1, sum(self.recv_units)), 4), dtype=torch.int32, device=dev)

    def exchange(self) -> None:
        if self.nranks > 1:
            exchange_units(self._send, self._recv, self.send_units, self.recv_units, self.group)

    def _agree(self, rc: int, what: str) -> None:
        """Every rank learns whether any rank failed `what`, and all raise together
        (a rank that raised alone would leave its peers waiting in the exchange or
        in gathered_results' all-reduce)."""
        import torch
        import torch.distributed as dist
        if self.nranks == 1 and not dist.is_initialized():   # one rank, no process group
            self._check(rc)
            return
        flag = torch.tensor([1 if rc else 0], dtype=torch.int32)
        if dist.get_backend(self.group) == "nccl":
            flag = flag.cuda(self.cfg.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        self._check(rc)
        if int(flag.item()):
            raise GnocError(-3, f"{what} failed on another rank")

    def run(self) -> None:
        self._agree(self.lib.gnoc_run_begin(self._h, self._send.data_ptr()), "gnoc_run_begin")
        self.exchange()
        self._agree(self.lib.gnoc_run_finish(self._h, self._recv.data_ptr()), "gnoc_run_finish")

    def gathered_results(self) -> Results:
        """The whole mesh's results on every rank: element-wise sum over ranks
        (each entry is non-zero on the one rank that owns it)."""
        import torch
        import torch.distributed as dist
        r = self.results()
        if self.nranks == 1 and not dist.is_initialized():
            return r
        parts = [r.final_ps, r.zero_load_ps, r.contention_ps, r.port_sum_delay, r.port_count, r.port_mg1,
                 r.port_flit, r.port_last]
        flat = torch.from_numpy(np.concatenate(parts).view(np.int64).copy())
        if dist.get_backend(self.group) == "nccl":
            flat = flat.cuda(self.cfg.device)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        out = flat.cpu().numpy().view(np.uint64)
        n, npt = self._n, r.port_sum_delay.shape[0]
        o = [0, n, 2 * n, 3 * n, 3 * n + npt, 3 * n + 2 * npt, 3 * n + 3 * npt, 3 * n + 4 * npt, 3 * n + 5 * npt]
        a = [out[o[k]:o[k + 1]].copy() for k in range(8)]
        return Results(*a[:6], summary=r.summary, port_flit=a[6], port_last=a[7])


RCCL_ID_BYTES = 128   # GNOC_RCCL_ID_BYTES


class RcclComm:
    """An RCCL communicator made by libgnoc's own RCCL (gnoc_rccl_comm_init), for
    gnoc_shard_set_comm.  The 128-byte unique id goes from rank 0 to every rank
    over `broadcast(buf: bytearray)` -- by default torch.distributed's default
    process group (any backend)."""

    def __init__(self, nranks: int, rank: int, device: int, broadcast=None):
        self.lib = load()
        idb = (ctypes.c_ubyte * RCCL_ID_BYTES)()
        if rank == 0:
            rc = self.lib.gnoc_rccl_unique_id(ctypes.cast(idb, ctypes.c_void_p))
            if rc:
                raise GnocError(rc, "ncclGetUniqueId failed")
        if nranks > 1:
            buf = bytearray(bytes(idb))
            (broadcast or _torch_broadcast_bytes)(buf)
            ctypes.memmove(idb, bytes(buf), RCCL_ID_BYTES)
        self.comm = ctypes.c_void_p()
        rc = self.lib.gnoc_rccl_comm_init(nranks, rank, device, ctypes.cast(idb, ctypes.c_void_p), ctypes.byref(self.comm))
        if rc:
            raise GnocError(rc, "ncclCommInitRank failed")

    def close(self) -> None:
        if self.comm:
            self.lib.gnoc_rccl_comm_destroy(self.comm)
            self.comm = ctypes.c_void_p()


def _torch_broadcast_bytes(buf: bytearray) -> None:
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(buf), dtype=torch.uint8)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.broadcast(t, 0)
    buf[:] = bytes(t.cpu().tolist())


class NativeShardedEngine(Engine):
    """One rank's share of a sharded mesh with the exchange inside libgnoc:
    gnoc_shard + gnoc_shard_set_comm(an RcclComm) + gnoc_run_sharded (prep and X
    phase, grouped ncclSend / ncclRecv of the turn records over xGMI on the
    engine's stream, Y phase; every rank's status max-reduced around the
    exchange).  No torch collective and no Python on the data path."""

    def __init__(self, cfg: EngineConfig, rank: int, nranks: int, comm: RcclComm):
        super().__init__(cfg)
        self.rank, self.nranks, self.comm_obj = rank, nranks, comm
        self._check(self.lib.gnoc_shard(self._h, rank, nranks))
        self._check(self.lib.gnoc_shard_set_comm(self._h, comm.comm))

    def run(self) -> None:
        self._check(self.lib.gnoc_run_sharded(self._h))

    group = None
    gathered_results = ShardedEngine.gathered_results


class LocalShardSet:
    """Every rank of a sharded mesh in ONE process on one device: the same
    gnoc_shard engines and device kernels as a multi-GPU run, with the
    all-to-all done by copies between the ranks' buffers.  For parity tests of
    any rank count on a single GPU, and for per-rank device timings."""

    def __init__(self, cfg: EngineConfig, nranks: int):
        self.cfg, self.n = cfg, nranks
        self.engs = []
        for r in range(nranks):
            e = Engine(cfg)
            e._check(e.lib.gnoc_shard(e._h, r, nranks))
            self.engs.append(e)

    def submit(self, tr: Trace) -> None:
        import torch
        dev = torch.device("cuda", self.cfg.device)
        self.su, self.ru, self.send, self.recv = [], [], [], []
        for e in self.engs:
            e.submit(tr)
            s = np.zeros(self.n, np.uint64)
            r = np.zeros(self.n, np.uint64)
            e._check(e.lib.gnoc_exchange_counts(e._h, s.ctypes.data, r.ctypes.data, self.n))
            self.su.append([int(v) for v in s])
            self.ru.append([int(v) for v in r])
            self.send.append(torch.empty((max(1, int(s.sum())), 4), dtype=torch.int32, device=dev))
            self.recv.append(torch.empty((max(1, int(r.sum())), 4), dtype=torch.int32, device=dev))

    def exchange(self) -> None:
        import torch
        for d in range(self.n):
            o = 0
            for r in range(self.n):
                k = self.ru[d][r]
                assert k == self.su[r][d], "send/receive sizes disagree"
                so = sum(self.su[r][:d])
                self.recv[d][o:o + k].copy_(self.send[r][so:so + k])
                o += k
        torch.cuda.synchronize()

    def run(self) -> None:
        for e, s in zip(self.engs, self.send):
            e._check(e.lib.gnoc_run_begin(e._h, s.data_ptr()))
        self.exchange()
        for e, r in zip(self.engs, self.recv):
            e._check(e.lib.gnoc_run_finish(e._h, r.data_ptr()))

    def results(self) -> Results:
        """Whole-mesh results: element-wise sum over ranks."""
        rs = [e.results() for e in self.engs]
        f = lambda k: np.sum([getattr(r, k) for r in rs], axis=0, dtype=np.uint64)
        return Results(f("final_ps"), f("zero_load_ps"), f("contention_ps"), f("port_sum_delay"), f("port_count"),
                       f("port_mg1"), rs[0].summary, f("port_flit"), f("port_last"))

    def set_profiling(self, on: bool) -> None:
        for e in self.engs:
            e.set_profiling(on)

    def close(self) -> None:
        for e in self.engs:
            e.close()


# ---------------------------------------------------------------------------
# design-space sweep (gnoc_create_sweep)
# ---------------------------------------------------------------------------
@dataclass
class SweepPoint:
    """The per-point carbon_sim.cfg keys a sweep varies."""
    flit_width: int = 64
    router_delay: int = 1
    link_delay: int = 1
    tile_width_mm: float = 1.0

    def config(self, base: EngineConfig) -> EngineConfig:
        """This point as a stand-alone engine / oracle configuration."""
        from dataclasses import replace
        return replace(base, flit_width=self.flit_width, router_delay=self.router_delay,
                       link_delay=self.link_delay, tile_width_mm=self.tile_width_mm)


def sweep_global_tile(p, t, W, H, bx):
    """G(p, t) of include/gnoc.h: local tile t of point p in the blocks_x-wide block grid."""
    p = np.asarray(p, np.int64)
    t = np.asarray(t, np.int64)
    return ((p // bx) * H + t // W) * (bx * W) + (p % bx) * W + t % W


def sweep_merge(traces, W, H, bx):
    """(merged Trace with global tiles, order): the (inject_ps, point, id)-ordered
    merge; order[k] = (point, local id) of merged packet k as two arrays."""
    pts = np.concatenate([np.full(len(t), i, np.int64) for i, t in enumerate(traces)]) if traces else np.zeros(0, np.int64)
    lid = np.concatenate([np.arange(len(t), dtype=np.int64) for t in traces]) if traces else np.zeros(0, np.int64)
    trs = [t.normalized() for t in traces]
    inj = np.concatenate([t.inject_ps for t in trs]) if trs else np.zeros(0, np.uint64)
    order = np.lexsort((lid, pts, inj))
    p, l = pts[order], lid[order]
    src = np.concatenate([t.src for t in trs])[order] if trs else np.zeros(0, np.uint32)
    dst = np.concatenate([t.dst for t in trs])[order] if trs else np.zeros(0, np.uint32)
    bits = np.concatenate([t.bits for t in trs])[order] if trs else np.zeros(0, np.uint32)
    flags = np.concatenate([t.flags for t in trs])[order] if trs else np.zeros(0, np.uint32)
    merged = Trace(inj[order], sweep_global_tile(p, src, W, H, bx).astype(np.uint32),
                   sweep_global_tile(p, dst, W, H, bx).astype(np.uint32), bits, flags)
    return merged, (p, l)


class SweepEngine:
    """Many independent design points timed in one batch on one GPU (one engine
    per rank; ranks take disjoint slices of the points -- no collective)."""

    def __init__(self, base: EngineConfig, points):
        self.lib = load()
        self.base, self.points = base, list(points)
        self.W, self.H = base.width, base.height
        arr = (GnocPoint * len(self.points))(*[GnocPoint(q.flit_width, q.router_delay, q.link_delay, q.tile_width_mm)
                                                for q in self.points])
        self._h = ctypes.c_void_p()
        c = base.to_c()
        rc = self.lib.gnoc_create_sweep(ctypes.byref(c), arr, len(self.points), ctypes.byref(self._h))
        if rc:
            raise GnocError(rc, "gnoc_create_sweep rejected the configuration")
        bx, by = ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.gnoc_sweep_layout(self._h, ctypes.byref(bx), ctypes.byref(by)))
        self.bx, self.by = bx.value, by.value
        self._n = 0

    _check = Engine._check
    close = Engine.close
    run = Engine.run
    summary = Engine.summary
    set_profiling = Engine.set_profiling
    kernel_stats = Engine.kernel_stats

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def submit(self, traces) -> None:
        assert len(traces) == len(self.points)
        merged, (self._pt, self._lid) = sweep_merge(traces, self.W, self.H, self.bx)
        self._counts = [len(t) for t in traces]
        tr = merged.normalized()
        pk = GnocPackets(tr.inject_ps.ctypes.data, tr.src.ctypes.data, tr.dst.ctypes.data, tr.bits.ctypes.data,
                         tr.flags.ctypes.data)
        self._check(self.lib.gnoc_submit(self._h, ctypes.byref(pk), len(tr)))
        self._n = len(tr)

    def results(self):
        """One Results per point, in the point's own packet and port numbering."""
        n = self._n
        fin, zl, ct = (np.empty(n, np.uint64) for _ in range(3))
        self._check(self.lib.gnoc_get_packet_results(self._h, fin.ctypes.data, zl.ctypes.data, ct.ctypes.data, n))
        npt = self.bx * self.W * self.by * self.H * PORTS_PER_TILE
        ps, pc, pm = (np.empty(npt, np.uint64) for _ in range(3))
        self._check(self.lib.gnoc_get_port_stats(self._h, ps.ctypes.data, pc.ctypes.data, pm.ctypes.data, npt))
        pf, pl = np.empty(npt, np.uint64), np.empty(npt, np.uint64)
        self._check(self.lib.gnoc_get_port_utilization(self._h, pf.ctypes.data, pl.ctypes.data, npt))
        out = []
        tiles = np.arange(self.W * self.H)
        for p, cnt in enumerate(self._counts):
            m = self._pt == p
            idx = np.empty(cnt, np.int64)
            idx[self._lid[m]] = np.nonzero(m)[0]
            g = (sweep_global_tile(p, tiles, self.W, self.H, self.bx)[:, None] * PORTS_PER_TILE +
                 np.arange(PORTS_PER_TILE)[None, :]).reshape(-1)
            out.append(Results(fin[idx], zl[idx], ct[idx], ps[g], pc[g], pm[g], {}, pf[g], pl[g]))
        return out
