import sys
sys.path.insert(0, ".")
import numpy as np
from graphite_amd import gnoc
base = gnoc.synthetic_trace(32, 32, 0.005, 10000, seed=1)
rng = np.random.default_rng(7)
rng.random(len(base))
tr = gnoc.Trace(base.inject_ps, base.src, base.dst, base.bits, base.flags.copy())
tr.flags[rng.random(len(tr)) < 1e-4] |= gnoc.PKT_BROADCAST
bi = np.nonzero(tr.flags & gnoc.PKT_BROADCAST)[0]
np.savetxt("gpurun_out/bcast_ids.txt", np.stack([bi, tr.inject_ps[bi], tr.src[bi]], 1), fmt="%d")
eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
eng.submit(tr)
eng.run()
print(eng.broadcast_info())
