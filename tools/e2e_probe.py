"""Where the pipelined end-to-end time goes (configs[1]): runs alone, runs with only the
read-backs pipelined, runs with only the uploads pipelined, both, and the bare copies."""
import sys
import time
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from graphite_amd import gnoc          # noqa: E402
from bench import pinned_array         # noqa: E402

K = 10
tr = gnoc.synthetic_trace(32, 32, 0.005, 10000, seed=1)
cfg = gnoc.EngineConfig(num_tiles=1024)
eng = gnoc.Engine(cfg)
ntr = gnoc.NarrowTrace.of(tr, alloc=lambda shape, dt: pinned_array(shape[0], dt))
ktr = gnoc.PackedTrace.of(tr, alloc=lambda shape, dt: pinned_array(shape[0], dt))
fins = [pinned_array(len(tr), np.uint64) for _ in range(2)]
lats = [pinned_array(len(tr), np.uint32) for _ in range(2)]
eng.submit_narrow(ntr)
for _ in range(5):
    eng.run()
for _ in range(2):
    eng.submit_async_narrow(ntr)
    eng.submit_commit()
    eng.run()
    eng.fetch_final_ps(fins[0])
    eng.fetch_wait()
    eng.run()
    eng.fetch_latency(lats[0])
    eng.fetch_wait()
print("trace bytes per packet (narrow wire):", sum(getattr(ntr, f).itemsize for f in ntr.__dataclass_fields__) if hasattr(ntr, "__dataclass_fields__") else "?")


def clock(name, body):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(K):
        body(k)
    eng.fetch_wait()
    torch.cuda.synchronize()
    print(f"{name:28s} {(time.perf_counter() - t) / K * 1e3:7.3f} ms", flush=True)


def run_only(k):
    eng.run()


def run_fetch(k):
    eng.run()
    eng.fetch_final_ps(fins[k % 2])


def run_upload(k):
    eng.submit_async_narrow(ntr)
    eng.run()
    eng.submit_commit()


def full(k):
    eng.submit_async_narrow(ntr)
    eng.run()
    eng.fetch_final_ps(fins[k % 2])
    eng.submit_commit()


def run_lat(k):
    eng.run()
    eng.fetch_latency(lats[k % 2])


def full_lat(k):
    eng.submit_async_narrow(ntr)
    eng.run()
    eng.fetch_latency(lats[k % 2])
    eng.submit_commit()


def lat_only(k):
    eng.fetch_latency(lats[k % 2])
    eng.fetch_wait()


def run_upk(k):
    eng.submit_async_packed(ktr)
    eng.run()
    eng.submit_commit()


def full_pk(k):
    eng.submit_async_packed(ktr)
    eng.run()
    eng.fetch_latency(lats[k % 2])
    eng.submit_commit()


def upk_only(k):
    eng.submit_async_packed(ktr)
    eng.submit_commit()
    torch.cuda.synchronize()


def fetch_only(k):
    eng.fetch_final_ps(fins[k % 2])
    eng.fetch_wait()


def upload_only(k):
    eng.submit_async_narrow(ntr)
    eng.submit_commit()
    torch.cuda.synchronize()


def submit_serial(k):
    eng.submit_narrow(ntr)


for name, body in (("run", run_only), ("run + fetch (pipelined)", run_fetch), ("fetch alone", fetch_only),
                   ("run + latency (pipelined)", run_lat), ("latency alone", lat_only),
                   ("run + upload (pipelined)", run_upload), ("run + upload + fetch", full),
                   ("run + upload + latency", full_lat), ("upload+commit alone", upload_only),
                   ("run + packed upload", run_upk), ("run + packed upload + latency", full_pk),
                   ("packed upload+commit alone", upk_only),
                   ("submit_narrow alone", submit_serial), ("run", run_only), ("fetch alone", fetch_only)):
    clock(name, body)
eng.close()
