"""Dev tool: locate the first divergence between the GPU engine and the oracle
on one trace (default: the saturated 8x8 M/G/1 case).  Prints the earliest
mismatching ports in level order and the packets through them."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402
from oracle import oracle  # noqa: E402
from tests.traces import random_trace  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
burst = int(sys.argv[2]) if len(sys.argv) > 2 else 400
W = 8
cfg = gnoc.EngineConfig(num_tiles=W * W)
tr = random_trace(n, W, W, seed=3, max_cycle=300, burst0=burst)
e = gnoc.Engine(cfg)
e.submit(tr)
e.run()
got = e.results()
ref = oracle.run(cfg, tr)
print("summary", got.summary, "oracle mg1", int(ref.port_mg1.sum()))
names = ["SELF", "LEFT", "RIGHT", "DOWN", "UP", "INJ"]
bad = np.nonzero((got.port_sum_delay != ref.port_sum_delay) | (got.port_count != ref.port_count) |
                 (got.port_mg1 != ref.port_mg1))[0]
print("bad ports", bad.size)


def level(p):
    t, d = divmod(int(p), 6)
    x, y = t % W, t // W
    if d == 5: return 0
    if d == 2: return 1 + x
    if d == 1: return W - x
    if d == 4: return W + y
    if d == 3: return W + (W - 1 - y)
    return 2 * W - 1


for p in sorted(bad, key=level)[:8]:
    t, d = divmod(int(p), 6)
    print(f"port {p} tile {t} ({t % W},{t // W}) {names[d]} level {level(p)}: sum {got.port_sum_delay[p]} vs {ref.port_sum_delay[p]}"
          f" cnt {got.port_count[p]} vs {ref.port_count[p]} mg1 {got.port_mg1[p]} vs {ref.port_mg1[p]}")
fb = np.nonzero(got.final_ps != ref.final_ps)[0]
print("bad packets", fb.size)
for i in fb[:5]:
    print(f"  pkt {i} t={tr.inject_ps[i]} src {tr.src[i]} dst {tr.dst[i]} gpu {got.final_ps[i]} ref {ref.final_ps[i]}")
