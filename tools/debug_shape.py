"""Dev tool: first divergence between the engine and the oracle on
test_gpu_parity's mesh-shape batch (W H [seed]): the mismatching ports in
level order, the packets through them, and the engine's summary."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.traces import random_trace  # noqa: E402

W, H = int(sys.argv[1]), int(sys.argv[2])
cfg = gnoc.EngineConfig(num_tiles=W * H, mesh_width=W, mesh_height=H)
tr = random_trace(3000, W, H, seed=W * 10 + H, max_cycle=400, burst0=50, self_frac=0.05)
ref = oracle.run(cfg, tr)
e = gnoc.Engine(cfg)
e.submit(tr)
names = ["SELF", "LEFT", "RIGHT", "DOWN", "UP", "INJ"]
for run in range(2):
    e.run()
    got = e.results()
    print("run", run, "summary", got.summary, "oracle mg1", int(ref.port_mg1.sum()))
    bad = np.nonzero((got.port_sum_delay != ref.port_sum_delay) | (got.port_count != ref.port_count) |
                     (got.port_mg1 != ref.port_mg1))[0]
    print("bad ports", bad.size)
    for p in bad[:12]:
        t, d = divmod(int(p), 6)
        print(f"port {p} tile {t} ({t % W},{t // W}) {names[d]}: sum {got.port_sum_delay[p]} vs {ref.port_sum_delay[p]}"
              f" cnt {got.port_count[p]} vs {ref.port_count[p]} mg1 {got.port_mg1[p]} vs {ref.port_mg1[p]}"
              f" last {got.port_last[p]} vs {ref.port_last[p]}")
    fb = np.nonzero(got.final_ps != ref.final_ps)[0]
    print("bad packets", fb.size)
    for i in fb[:6]:
        print(f"  pkt {i} t={tr.inject_ps[i]} src {tr.src[i]} dst {tr.dst[i]} gpu {got.final_ps[i]} ref {ref.final_ps[i]}")
e.close()
