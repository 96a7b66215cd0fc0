"""One rank of a sharded run (gnoc_shard), launched by tests/test_gpu_shard.py as
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... tests/shard_worker.py CASE...
Every rank drives the same GPU (the test box has one) over the gloo backend, so
the turn exchange is staged through host memory; on a multi-GPU node the same
ShardedEngine exchanges over RCCL.  Rank 0 checks the gathered whole-mesh
results bit-exactly against the oracle (small cases) or an unsharded run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from graphite_amd import gnoc  # noqa: E402
from tests.traces import random_trace  # noqa: E402


def case(name):
    if name == "syn8":
        return gnoc.EngineConfig(num_tiles=64), gnoc.synthetic_trace(8, 8, 0.05, 300, seed=11), "oracle"
    if name == "sat8":   # M/G/1 exceptions produced in the X phase cross ranks
        return gnoc.EngineConfig(num_tiles=64), random_trace(20000, 8, 8, seed=3, max_cycle=300, burst0=400), "oracle"
    if name == "shape6":  # uneven bands, self-sends, unmodeled packets
        return (gnoc.EngineConfig(num_tiles=36),
                random_trace(6000, 6, 6, seed=66, max_cycle=400, burst0=50, self_frac=0.05, unmodeled_frac=0.05),
                "oracle")
    if name == "rect":    # W != H
        return (gnoc.EngineConfig(num_tiles=24, mesh_width=6, mesh_height=4),
                random_trace(5000, 6, 4, seed=64, max_cycle=300, burst0=30), "oracle")
    if name == "nocont":
        return (gnoc.EngineConfig(num_tiles=16, contention_enabled=False),
                random_trace(3000, 4, 4, seed=9, max_cycle=300, self_frac=0.1), "oracle")
    if name == "m32":
        return gnoc.EngineConfig(num_tiles=1024), gnoc.synthetic_trace(32, 32, 0.005, 300, seed=5), "engine"
    if name == "m32hot":
        return (gnoc.EngineConfig(num_tiles=1024),
                gnoc.synthetic_trace(32, 32, 0.01, 200, seed=6, hotspot_fraction=0.2, num_hotspots=16), "engine")
    raise ValueError(name)


def same(a, b):
    for k in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
        x, y = getattr(a, k), getattr(b, k)
        if not np.array_equal(x, y):
            bad = np.nonzero(x != y)[0]
            return f"{k}: {bad.size} differ, first {bad[0]}: sharded {x[bad[0]]} expected {y[bad[0]]}"
    return None


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    failures = 0
    for name in sys.argv[1:]:
        if name == "fail":
            # rank 1's X phase fails: every rank must raise (none may hang in the exchange)
            os.environ["GNOC_FAIL_RANK"] = "1"
            eng = gnoc.ShardedEngine(gnoc.EngineConfig(num_tiles=64), rank, world)
            eng.submit(gnoc.synthetic_trace(8, 8, 0.05, 100, seed=11))
            try:
                eng.run()
                raised = False
            except gnoc.GnocError:
                raised = True
            os.environ.pop("GNOC_FAIL_RANK")
            eng.close()
            flag = torch.tensor([1 if raised else 0], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if rank == 0:
                if int(flag.item()) == 1:
                    print(f"SHARD OK {name} world={world}", flush=True)
                else:
                    failures += 1
                    print(f"SHARD FAIL {name} world={world}: a rank did not raise", flush=True)
            continue
        cfg, tr, ref_kind = case(name)
        eng = gnoc.ShardedEngine(cfg, rank, world)
        eng.submit(tr)
        eng.run()
        eng.run()   # twice: per-run state is reset
        got = eng.gathered_results()
        eng.close()
        if rank == 0:
            if ref_kind == "oracle":
                from oracle import oracle
                ref = oracle.run(cfg, tr)
            else:
                e1 = gnoc.Engine(cfg)
                e1.submit(tr)
                e1.run()
                ref = e1.results()
                e1.close()
            err = same(got, ref)
            mg1 = int(ref.port_mg1.sum())
            if err:
                failures += 1
                print(f"SHARD FAIL {name} world={world}: {err}", flush=True)
            else:
                print(f"SHARD OK {name} world={world} packets={len(tr)} mg1={mg1}", flush=True)
        dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if failures else 0)


if __name__ == "__main__":
    main()
