"""Run configs[1] (32x32, load 0.005, 10,000 packets per tile) a few times on the
library GNOC_LIB names and print the per-run ms (for rocprofv3 kernel traces of
timing variants).

    python tools/run_probe.py [runs] [hotspot_fraction]

GNOC_PROBE_PROF=1 adds one profiled run's per-kernel-class device ms.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    hot = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    tr = gnoc.synthetic_trace(32, 32, 0.005, 10000, seed=1, hotspot_fraction=hot, num_hotspots=16)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
    eng.submit(tr)
    ms = []
    for _ in range(runs):
        eng.run()
        ms.append(round(eng.summary()["last_run_ms"], 3))
    s = eng.summary()
    print("lib", os.environ.get("GNOC_LIB", "default"), "path", s["engine_path"], "ms", ms,
          "windows", s.get("windows"), s.get("windows_y"), "reruns", s.get("retries_total"), s.get("fallbacks_total"),
          flush=True)
    if os.environ.get("GNOC_PROBE_PROF"):
        eng.set_profiling(True)
        eng.run()
        print("kernel_ms", {k: round(v[0], 4) for k, v in eng.kernel_stats().items() if v[1]}, flush=True)
    eng.close()


if __name__ == "__main__":
    main()
