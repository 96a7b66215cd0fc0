"""configs[1] behind a cycle-0 burst (tests/golden/make_fullsize.py's
32x32_burst4 case: M/G/1 requests in injection and mesh ports): settled run time
and engine path on the default engine (the chains' MG instantiation) and, for
comparison, on the level engine (GNOC_ENGINE=levels).  Dev tool, not a test."""
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(label):
    import torch  # noqa: F401
    from graphite_amd import gnoc
    from tests.golden.make_fullsize import trace_of
    tr = trace_of("32x32_burst4_l0.005_ppt10000")
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
    eng.submit(tr)
    for _ in range(4):
        eng.run()
    K = 10
    t = time.perf_counter()
    for _ in range(K):
        eng.run()
    ms = (time.perf_counter() - t) / K * 1e3
    s = eng.summary()
    print(label, f"{ms:.3f} ms/run", {k: s[k] for k in ("engine_path", "chain_protocol", "mg1_uses", "retries",
                                                         "fallbacks", "mesh_hops", "windows", "windows_y",
                                                         "window_ps_x", "window_ps_y")}, flush=True)
    eng.set_profiling(True)
    eng.run()
    print(label, "kernel_ms", {k: round(v[0], 4) for k, v in eng.kernel_stats().items()}, flush=True)
    eng.close()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        one(sys.argv[1])
    else:
        for label, env in (("chains", {}), ("levels", {"GNOC_ENGINE": "levels"})):
            subprocess.run([sys.executable, __file__, label], env={**os.environ, **env}, check=True)
