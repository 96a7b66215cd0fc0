"""Host side of the sharded mesh (gnoc_shard), on CPU: the band split, the turn
counts the exchange sizes come from, and the all-to-all of 16-byte units over a
world-size-2 gloo group (the same exchange_units a multi-GPU run uses over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from graphite_amd import gnoc
from tests.traces import random_trace


def test_bands_partition():
    for dim in (4, 6, 7, 32, 64):
        for n in range(1, min(dim, 8) + 1):
            cover = [i for b in range(n) for i in gnoc.band(b, n, dim)]
            assert cover == list(range(dim))
            sizes = [len(gnoc.band(b, n, dim)) for b in range(n)]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("W,H,n", [(8, 8, 2), (6, 6, 4), (6, 4, 3), (32, 32, 8)])
def test_turn_counts_one_per_routed_packet(W, H, n):
    tr = random_trace(5000, W, H, seed=W + n, self_frac=0.05, unmodeled_frac=0.05)
    m = gnoc.turn_counts(tr, W, H, n)
    routed = (tr.src != tr.dst) & ((tr.flags & gnoc.PKT_UNMODELED) == 0)
    assert m.sum() == routed.sum()
    # the turn record sits at tile (dx, sy): row band of the source, column band of the destination
    sy, dx = tr.src[routed] // W, tr.dst[routed] % W
    for r in range(n):
        for d in range(n):
            rows, cols = gnoc.band(r, n, H), gnoc.band(d, n, W)
            want = np.sum((sy >= rows.start) & (sy < rows.stop) & (dx >= cols.start) & (dx < cols.stop))
            assert m[r, d] == want


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = gnoc.turn_counts(random_trace(4000, 8, 8, seed=2), 8, 8, world)
        # per pair: a status unit, then the exception counts (u32 per turn slot, 9 per tile)
        hdr = lambda r, d: 1 + (len(gnoc.band(r, world, 8)) * len(gnoc.band(d, world, 8)) * 9 + 3) // 4
        su = [0 if d == rank else hdr(rank, d) + int(m[rank, d]) for d in range(world)]
        ru = [0 if r == rank else hdr(r, rank) + int(m[r, rank]) for r in range(world)]
        # unit k of the block for peer d carries (rank, d, k) so the receiver can check provenance
        send = torch.zeros((sum(su), 4), dtype=torch.int32)
        o = 0
        for d in range(world):
            for k in range(su[d]):
                send[o] = torch.tensor([rank, d, k, 7], dtype=torch.int32)
                o += 1
        recv = torch.full((sum(ru), 4), -1, dtype=torch.int32)
        gnoc.exchange_units(send, recv, su, ru)
        o, ok = 0, True
        for r in range(world):
            for k in range(ru[r]):
                ok &= recv[o].tolist() == [r, rank, k, 7]
                o += 1
        q.put((rank, ok, sum(su), sum(ru)))
    finally:
        dist.destroy_process_group()


def test_exchange_units_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res
    # what rank 0 sends is what rank 1 receives and vice versa
    assert res[0][2] == res[1][3] and res[1][2] == res[0][3]
