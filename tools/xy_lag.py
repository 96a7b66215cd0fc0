"""Fused X+Y launch: step time on configs[1] (uniform and hotspot) for several Y
task lags (GNOC_XY_LAG, in units of the batch's last injection time)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402


def main():
    lags = [float(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0.2", "0.3", "0.4", "0.5"])]
    ppt = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    for hot in (0.0, 0.2):
        tr = gnoc.synthetic_trace(32, 32, 0.005, ppt, seed=1, hotspot_fraction=hot, num_hotspots=16)
        for lag in lags:
            os.environ["GNOC_XY_LAG"] = str(lag)
            e = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
            e.submit(tr)
            fused, sep = [], []
            for _ in range(14):
                e.run()
                s = e.summary()
                (fused if s["chain_protocol"] & 0x200 else sep).append(s["last_run_ms"])
            e.set_profiling(True)
            e.run()
            ks = e.kernel_stats()
            e.set_profiling(False)
            e.close()
            print(f"hot {hot} lag {lag}: fused min {min(fused) if fused else 0:.3f} med "
                  f"{sorted(fused)[len(fused) // 2] if fused else 0:.3f} ms ({len(fused)} runs) | separate min "
                  f"{min(sep) if sep else 0:.3f} | proto {s['chain_protocol']:#x} | k_chain {ks.get('k_chain', (0, 0))}",
                  flush=True)


if __name__ == "__main__":
    main()
