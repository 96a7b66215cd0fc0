"""Dev tool: test_rccl_declined_x_phase_poisons_and_reruns step by step (1-rank
RCCL communicator, self exchange, one injected X decline): each run's summary."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc  # noqa: E402
from oracle import oracle  # noqa: E402

os.environ.setdefault("GNOC_SHARD_SELF_EXCHANGE", "1")
os.environ.setdefault("GNOC_DECLINE_ONCE_RANK", "0")
cfg = gnoc.EngineConfig(num_tiles=64)
tr = gnoc.synthetic_trace(8, 8, 0.05, 300, seed=13)
ref = oracle.run(cfg, tr)
print("oracle mg1", int(ref.port_mg1.sum()), "per dir", ref.port_mg1.reshape(-1, 6).sum(0))
comm = gnoc.RcclComm(1, 0, 0)
eng = gnoc.NativeShardedEngine(cfg, 0, 1, comm)
eng.submit(tr)
for k in range(5):
    eng.run()
    s = eng.summary()
    got = eng.results()
    print(k, {q: s[q] for q in ("engine_path", "retries", "fallbacks", "runs", "chain_protocol", "mg1_uses")},
          "exact", bool(np.array_equal(got.final_ps, ref.final_ps)))
eng.close()
comm.close()
print("unsharded")
e = gnoc.Engine(cfg)
e.submit(tr)
for k in range(3):
    e.run()
    s = e.summary()
    print(k, {q: s[q] for q in ("engine_path", "retries", "fallbacks", "runs", "chain_protocol", "mg1_uses")},
          "exact", bool(np.array_equal(e.results().final_ps, ref.final_ps)))
e.close()
