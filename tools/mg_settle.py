"""Per-run engine path, chain protocol bits and time of the configs[1] burst batch
(the full-size M/G/1 pin's trace): on which run the MG instantiation (bit 10) and the
mixed launch (bit 11, only the M/G/1 windows on the MG path) start.  Dev tool."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402
from tests.golden.make_fullsize import trace_of  # noqa: E402

tr = trace_of("32x32_burst4_l0.005_ppt10000")
eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
eng.submit(tr)
for r in range(12):
    eng.run()
    s = eng.summary()
    print(f"run {r + 1}: path {s['engine_path']} protocol 0x{int(s['chain_protocol']):x} bit10 {int(s['chain_protocol']) >> 10 & 1} "
          f"bit11 {int(s['chain_protocol']) >> 11 & 1} retries {s['retries']} windows {s['windows']} {s['windows_y']} "
          f"ms {s['last_run_ms']:.2f}", flush=True)
eng.close()
