"""ctypes front-end of the CPU oracle (oracle/gnoc_oracle.c) and of the optional
reference build (oracle/_ref/libgnoc_ref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  The product (graphite_amd) never
imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libgnoc_ref.so")
REF_DIR = os.environ.get("GNOC_REF_DIR", "/root/reference")

_orc = None
_ref = None


def build(ref: bool | None = None) -> None:
    """make the oracle (and, when the reference tree exists here, oracle/_ref)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref is None:
        ref = os.path.isdir(REF_DIR)
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref", f"REF_DIR={REF_DIR}"], check=True)


def lib() -> ctypes.CDLL:
    global _orc
    if _orc is None:
        if not os.path.exists(ORACLE_SO):
            build(ref=False)
        L = ctypes.CDLL(ORACLE_SO)
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.orc_queue_create.restype = vp
        L.orc_queue_create.argtypes = [ctypes.c_int, ctypes.c_int, u64]
        L.orc_queue_compute.restype = u64
        L.orc_queue_compute.argtypes = [vp, u64, u64]
        L.orc_queue_mg1_uses.restype = u64
        L.orc_queue_mg1_uses.argtypes = [vp]
        L.orc_queue_size.argtypes = [vp]
        L.orc_queue_destroy.argtypes = [vp]
        L.orc_queue_destroy.restype = None
        L.orc_lat_to_ps.restype = u64
        L.orc_lat_to_ps.argtypes = [u64, ctypes.c_double]
        L.orc_time_to_cycles.restype = u64
        L.orc_time_to_cycles.argtypes = [u64, ctypes.c_double]
        L.orc_queue_create_type.restype = vp
        L.orc_queue_create_type.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, u64]
        L.orc_set_basic_moving_avg.argtypes = [ctypes.c_int, ctypes.c_uint32]
        L.orc_queue_set_moving_avg.argtypes = [vp, ctypes.c_int, ctypes.c_uint32]
        L.orc_ma_compute.restype = u64
        L.orc_ma_compute.argtypes = [vp, u64]
        L.orc_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u64, u64, ctypes.c_double, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t] + [vp] * 15
        _orc = L
    return _orc


def ref_lib() -> ctypes.CDLL | None:
    """The reference-compiled components, or None when not built (e.g. on the GPU box)."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO):
            return None
        L = ctypes.CDLL(REF_SO)
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.ref_queue_create.restype = vp
        L.ref_queue_create.argtypes = [ctypes.c_int, ctypes.c_int, u64]
        L.ref_queue_compute.restype = u64
        L.ref_queue_compute.argtypes = [vp, u64, u64]
        L.ref_queue_mg1_uses.restype = u64
        L.ref_queue_mg1_uses.argtypes = [vp]
        L.ref_queue_size.restype = ctypes.c_uint32
        L.ref_queue_size.argtypes = [vp]
        L.ref_queue_destroy.argtypes = [vp]
        L.ref_queue_destroy.restype = None
        L.ref_ma_create.restype = vp
        L.ref_ma_create.argtypes = [ctypes.c_int, ctypes.c_uint32]
        L.ref_ma_compute.restype = u64
        L.ref_ma_compute.argtypes = [vp, u64]
        L.ref_ma_destroy.argtypes = [vp]
        L.ref_ma_destroy.restype = None
        L.ref_lat_to_ps.restype = u64
        L.ref_lat_to_ps.argtypes = [u64, ctypes.c_double]
        L.ref_time_to_cycles.restype = u64
        L.ref_time_to_cycles.argtypes = [u64, ctypes.c_double]
        _ref = L
    return _ref


class Queue:
    """QueueModelHistoryTree / QueueModelHistoryList / QueueModelBasic
    (min_processing_time=1) restated (oracle).  kind: 0 history_tree, 1 basic
    (no moving average), 2 history_list."""

    def __init__(self, max_list_size: int = 100, analytical: bool = True, min_proc: int = 1, kind: int = 0,
                 interleaving: bool = True):
        self.L = lib()
        self.h = self.L.orc_queue_create_type(kind, max_list_size, int(analytical), int(interleaving), min_proc)
        if not self.h:
            raise ValueError("invalid queue model parameters")

    def set_moving_avg(self, ma_type: int, window: int) -> None:
        """QueueModelBasic with moving_avg_enabled (queue_model_basic.cc:7-30)."""
        if self.L.orc_queue_set_moving_avg(self.h, ma_type, window):
            raise ValueError("invalid moving average")

    def moving_avg(self, x: int) -> int:
        """MovingAverage::compute on the attached average alone (no queue update)."""
        return int(self.L.orc_ma_compute(self.h, x))

    def compute(self, t: int, p: int) -> int:
        return int(self.L.orc_queue_compute(self.h, t, p))

    @property
    def mg1_uses(self) -> int:
        return int(self.L.orc_queue_mg1_uses(self.h))

    def __del__(self):
        try:
            self.L.orc_queue_destroy(self.h)
        except Exception:
            pass


def run_hop_counter(cfg, tr) -> "OracleResult":
    """NetworkModelEMeshHopCounter restated (gnoc_oracle.c orc_run_hop_counter)."""
    L = lib()
    u64, vp = ctypes.c_uint64, ctypes.c_void_p
    L.orc_run_hop_counter.argtypes = [ctypes.c_int, ctypes.c_int, u64, u64, ctypes.c_double, ctypes.c_size_t] + [vp] * 8
    n = int(tr.inject_ps.shape[0])
    arrs = [np.ascontiguousarray(a, t) for a, t in ((tr.inject_ps, np.uint64), (tr.src, np.uint32),
                                                    (tr.dst, np.uint32), (tr.bits, np.uint32))]
    flags = np.ascontiguousarray(tr.flags if tr.flags is not None else np.zeros(n, np.uint32), np.uint32)
    fin, zl, ct = (np.zeros(n, np.uint64) for _ in range(3))
    rc = L.orc_run_hop_counter(cfg.num_tiles, cfg.flit_width, cfg.router_delay, cfg.link_delay, cfg.frequency_ghz, n,
                               *[a.ctypes.data for a in arrs], flags.ctypes.data, fin.ctypes.data, zl.ctypes.data,
                               ct.ctypes.data)
    if rc:
        raise ValueError(f"oracle rejected input (rc={rc})")
    z = np.zeros(0, np.uint64)
    return OracleResult(fin, zl, ct, z, z, z)


@dataclass
class OracleResult:
    final_ps: np.ndarray
    zero_load_ps: np.ndarray
    contention_ps: np.ndarray
    port_sum_delay: np.ndarray
    port_count: np.ndarray
    port_mg1: np.ndarray
    port_flit: np.ndarray = None     # QueueModel _total_utilized_cycles per port
    port_last: np.ndarray = None     # QueueModel _last_request_time per port
    # broadcast receipts: [broadcast (trace order), receiving tile]
    bcast_final_ps: np.ndarray = None
    bcast_zero_load_ps: np.ndarray = None


def run(cfg, tr, ref_queues: bool = False) -> OracleResult:
    """Event-driven reference walk of every packet (see gnoc_oracle.c).  cfg is a
    graphite_amd.gnoc.EngineConfig-like object, tr a Trace-like object.
    ref_queues: the history-tree queues are the reference's own IntervalTree and
    QueueModelMG1 objects (oracle/_ref, compiled from its sources; ref_driver.cc
    restates only computeQueueDelay's 80 lines over them) instead of the sorted-array
    restatement: bench.py's CPU baseline.  Needs oracle/_ref (ValueError otherwise)."""
    L = lib()
    if ref_queues:
        R = ref_lib()
        if R is None:
            raise ValueError("oracle/_ref is not built (needs /root/reference at build time)")
        vp = ctypes.c_void_p
        L.orc_set_queue_hooks.argtypes = [vp, vp, vp, vp]
        L.orc_set_queue_hooks(*(ctypes.cast(getattr(R, f), vp) for f in
                                ("ref_queue_create", "ref_queue_compute", "ref_queue_mg1_uses", "ref_queue_destroy")))
        try:
            return run(cfg, tr)
        finally:
            L.orc_set_queue_hooks(None, None, None, None)
    n = int(tr.inject_ps.shape[0])
    W, H = cfg.width, cfg.height
    inj = np.ascontiguousarray(tr.inject_ps, np.uint64)
    src = np.ascontiguousarray(tr.src, np.uint32)
    dst = np.ascontiguousarray(tr.dst, np.uint32)
    bits = np.ascontiguousarray(tr.bits, np.uint32)
    flags = np.ascontiguousarray(tr.flags if tr.flags is not None else np.zeros(n, np.uint32), np.uint32)
    fin, zl, ct = (np.zeros(n, np.uint64) for _ in range(3))
    npt = W * H * 6
    ps, pc, pm, pf, pl = (np.zeros(npt, np.uint64) for _ in range(5))
    nb = int(np.count_nonzero(flags & 2))
    bf, bz = (np.zeros((nb, W * H), np.uint64) for _ in range(2))
    ma = int(getattr(cfg, "moving_avg_type", 0)) if int(getattr(cfg, "queue_type", 0)) == 1 else 0
    if L.orc_set_basic_moving_avg(ma, int(getattr(cfg, "moving_avg_window", 1)) if ma else 1):
        raise ValueError("invalid moving average")
    rc = L.orc_run(W, H, cfg.flit_width, cfg.router_delay, cfg.link_delay, cfg.frequency_ghz,
                   int(cfg.contention_enabled), int(getattr(cfg, "queue_type", 0)),
                   int(getattr(cfg, "interleaving_enabled", True)), int(cfg.analytical_enabled), cfg.max_list_size, n,
                   inj.ctypes.data, src.ctypes.data, dst.ctypes.data, bits.ctypes.data, flags.ctypes.data,
                   fin.ctypes.data, zl.ctypes.data, ct.ctypes.data, ps.ctypes.data, pc.ctypes.data, pm.ctypes.data,
                   pf.ctypes.data, pl.ctypes.data, bf.ctypes.data if nb else None, bz.ctypes.data if nb else None)
    L.orc_set_basic_moving_avg(0, 1)
    if rc:
        raise ValueError(f"oracle rejected input (rc={rc})")
    return OracleResult(fin, zl, ct, ps, pc, pm, pf, pl, bf, bz)
