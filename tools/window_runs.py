"""Per-run chain-engine window behaviour on a repeated batch: device ms,
retries and fallbacks of each gnoc_run (adapted windows)."""
import sys

sys.path.insert(0, ".")
from graphite_amd import gnoc  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    load = float(sys.argv[2]) if len(sys.argv) > 2 else (0.002 if W == 64 else 0.005)
    runs = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    tr = gnoc.synthetic_trace(W, W, load, 10000, seed=1)
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=W * W))
    eng.submit(tr)
    for k in range(runs):
        eng.run()
        s = eng.summary()
        print(k, round(s["last_run_ms"], 3), "retries", s.get("retries"), "fallbacks", s.get("fallbacks"),
              s["window_ps_x"], s["window_ps_y"], flush=True)
    eng.close()


if __name__ == "__main__":
    main()
