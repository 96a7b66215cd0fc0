"""Regenerate the network-level golden vectors in tests/golden/*.npz.

Inputs: small seeded traces (tests/traces.py, and the synthetic_network
restatement in libgnoc).  Expected outputs: the CPU oracle (oracle/gnoc_oracle.c),
which is itself pinned by the reference's history_tree KAT and by differential
tests against the reference's compiled IntervalTree / QueueModelMG1 / time_types.h
(tests/test_oracle.py).  Run from the repo root:  python tests/golden/make_golden.py
"""
import dataclasses
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from graphite_amd import gnoc  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.traces import random_trace  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def case(name, cfg, tr):
    r = oracle.run(cfg, tr)
    d = {k: v for k, v in dataclasses.asdict(cfg).items()}
    np.savez_compressed(os.path.join(HERE, name + ".npz"), cfg=json.dumps(d), inject_ps=tr.inject_ps,
                        src=tr.src, dst=tr.dst, bits=tr.bits,
                        flags=tr.flags if tr.flags is not None else np.zeros(len(tr), np.uint32),
                        final_ps=r.final_ps, zero_load_ps=r.zero_load_ps, contention_ps=r.contention_ps,
                        port_sum_delay=r.port_sum_delay, port_count=r.port_count, port_mg1=r.port_mg1)
    print(name, len(tr), "mg1", int(r.port_mg1.sum()))


def main(only=None):
    E = gnoc.EngineConfig
    global case
    if only:
        full = case
        case = lambda name, cfg, tr: full(name, cfg, tr) if name.startswith(only) else None  # noqa: E731
    case("g_4x4_burst_mg1", E(num_tiles=16), random_trace(1500, 4, 4, seed=1, max_cycle=200, burst0=60))
    case("g_8x8_synthetic_0p05", E(num_tiles=64), gnoc.synthetic_trace(8, 8, 0.05, 60, seed=3))
    case("g_8x8_saturated", E(num_tiles=64), random_trace(4000, 8, 8, seed=2, max_cycle=150, burst0=100))
    case("g_4x4_self_unmodeled", E(num_tiles=16),
         random_trace(1500, 4, 4, seed=4, max_cycle=300, self_frac=0.2, unmodeled_frac=0.2))
    case("g_6x6_flit16_r2", E(num_tiles=36, flit_width=16, router_delay=2),
         random_trace(1500, 6, 6, seed=5, max_cycle=800, burst0=10, bits_choices=[72, 576, 584]))
    case("g_6x6_flit128_r0", E(num_tiles=36, flit_width=128, router_delay=0),
         random_trace(1500, 6, 6, seed=6, max_cycle=400, burst0=10, bits_choices=[72, 576, 1088]))
    case("g_4x4_link2", E(num_tiles=16, tile_width_mm=150.0, link_delay=2),
         random_trace(1500, 4, 4, seed=7, max_cycle=400, burst0=10))
    case("g_4x4_f0p9", E(num_tiles=16, frequency_ghz=0.9),
         random_trace(1500, 4, 4, seed=8, max_cycle=400, burst0=10, ps_jitter=True, frequency_ghz=0.9))
    case("g_4x4_list2", E(num_tiles=16, max_list_size=2), random_trace(1500, 4, 4, seed=9, max_cycle=200, burst0=30))
    case("g_2x4_noanalytical", E(num_tiles=8, analytical_enabled=False),
         random_trace(1000, 2, 4, seed=10, max_cycle=200, burst0=30))
    # queue_model/basic with its moving average (queue_model_basic.cc, moving_average.h);
    # the oracle's moving averages are pinned against the reference's header (test_oracle.py)
    case("g_4x4_basic_ma_arith_w8", E(num_tiles=16, queue_type=1, moving_avg_type=1, moving_avg_window=8),
         random_trace(1500, 4, 4, seed=11, max_cycle=300, burst0=20, self_frac=0.05, unmodeled_frac=0.05))
    case("g_4x4_basic_ma_median_w5", E(num_tiles=16, queue_type=1, moving_avg_type=3, moving_avg_window=5),
         random_trace(1500, 4, 4, seed=12, max_cycle=300, burst0=20))
    # geometric mean (moving_average.h:119-135, glibc pow): zeros in the window (the
    # mean becomes 0, then NaN), and a batch starting at cycle 1000 (finite means)
    case("g_4x4_basic_ma_geom_w6", E(num_tiles=16, queue_type=1, moving_avg_type=2, moving_avg_window=6),
         random_trace(1500, 4, 4, seed=13, max_cycle=300, burst0=20))
    late = random_trace(1500, 4, 4, seed=14, max_cycle=3000, burst0=20)
    late.inject_ps[:] += 1_000_000
    case("g_4x4_basic_ma_geom_w16_late", E(num_tiles=16, queue_type=1, moving_avg_type=2, moving_avg_window=16), late)


if __name__ == "__main__":
    import sys
    main(sys.argv[1] if len(sys.argv) > 1 else None)
