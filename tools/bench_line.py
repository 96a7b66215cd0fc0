"""One-line digest of a bench.py JSON line (uniform + hotspot)."""
import json
import sys

txt = open(sys.argv[1]).read().strip().splitlines()
d = json.loads([ln for ln in txt if ln.startswith("{")][-1])
tag = sys.argv[2] if len(sys.argv) > 2 else ""
km = {k: v for k, v in d["kernel_ms"].items() if v > 0.04}
print(tag, "uniform", round(d["ms_per_step"], 3), "ms", round(d["value"] / 1e9, 2), "G/s frac", round(d["roofline"]["frac"], 3),
      "chain_us", round(d["roofline"]["kernel_avg_us"], 1), d["reruns"], "settle", d.get("settle_runs"), d["config"]["windows"], km)
h = d.get("hotspot")
if h:
    print(tag, "hotspot", round(h["ms_per_step"], 3), "ms", round(h["value"] / 1e9, 2), "G/s frac", round(h["roofline_frac"], 3),
          "chain_us", round(h["kernel_avg_us"], 1), h["reruns"], {k: v for k, v in h["kernel_ms"].items() if v > 0.04})
