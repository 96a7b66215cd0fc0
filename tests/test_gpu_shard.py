"""One mesh sharded over several ranks (gnoc_shard, shard.hip): bit-exact
against the oracle and against the unsharded engine.  The box has one GPU, so
the ranks share it and exchange over gloo (host-staged); the device kernels,
the X/Y phase split and the turn-record layout are the ones an 8-GPU RCCL run
uses."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(nproc, cases, timeout=100):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "tests", "shard_worker.py")]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd + list(cases), cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    out = p.stdout + p.stderr
    print(out[-4000:])
    assert p.returncode == 0, out[-4000:]
    for c in cases:
        assert f"SHARD OK {c} world={nproc}" in out, out[-4000:]


def test_shard_two_ranks():
    launch(2, ["syn8", "sat8", "shape6", "rect", "nocont", "m32"])


def test_shard_four_ranks():
    launch(4, ["syn8", "sat8", "shape6", "rect", "m32hot"])


def test_shard_three_ranks_uneven():
    launch(3, ["shape6", "sat8"])


def test_shard_failure_on_one_rank_fails_every_rank():
    """One rank's X phase fails (GNOC_FAIL_RANK): the status all-reduce around the
    exchange makes every rank raise instead of waiting on the failed one."""
    launch(3, ["fail", "syn8"])


def _local_vs(cfg, tr, n, ref):
    from graphite_amd import gnoc
    import numpy as np
    ss = gnoc.LocalShardSet(cfg, n)
    ss.submit(tr)
    ss.run()
    ss.run()
    got = ss.results()
    ss.close()
    for k in ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit", "port_last"):
        a, b = getattr(got, k), getattr(ref, k)
        assert np.array_equal(a, b), f"{k} differs at {n} ranks: first {np.nonzero(a != b)[0][:5]}"


@pytest.mark.parametrize("n", [2, 5, 8])
def test_local_shards_vs_oracle_8x8_saturated(n):
    """All ranks in one process: M/G/1 tails from the X phase cross ranks."""
    from graphite_amd import gnoc
    from oracle import oracle
    from tests.traces import random_trace
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(20000, 8, 8, seed=3, max_cycle=300, burst0=400)
    ref = oracle.run(cfg, tr)
    assert ref.port_mg1.sum() > 0
    _local_vs(cfg, tr, n, ref)


@pytest.mark.parametrize("n", [3, 8])
def test_local_shards_vs_oracle_non_unit_frequency(n):
    """A sharded mesh at f = 0.9 GHz (the chunked path's double conversions on every rank)."""
    from graphite_amd import gnoc
    from oracle import oracle
    from tests.traces import random_trace
    cfg = gnoc.EngineConfig(num_tiles=64, frequency_ghz=0.9)
    tr = random_trace(20000, 8, 8, seed=5, max_cycle=2000, burst0=200, ps_jitter=True, frequency_ghz=0.9)
    ref = oracle.run(cfg, tr)
    _local_vs(cfg, tr, n, ref)


@pytest.mark.parametrize("W,n,hot", [(32, 8, 0.0), (32, 7, 0.2), (64, 8, 0.0)])
def test_local_shards_vs_unsharded(W, n, hot):
    from graphite_amd import gnoc
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    tr = gnoc.synthetic_trace(W, W, 0.005 if W == 32 else 0.002, 300 if W == 32 else 100, seed=4,
                              hotspot_fraction=hot, num_hotspots=16)
    e = gnoc.Engine(cfg)
    e.submit(tr)
    e.run()
    ref = e.results()
    e.close()
    _local_vs(cfg, tr, n, ref)


@pytest.mark.parametrize("bad", ["zero_flit", "too_long", "late"])
def test_bad_packet_on_one_rank_fails_every_rank(bad):
    """A packet that breaks the submit contract and that only rank 1 keeps (source
    in its row band, destination in its column band): every rank's gnoc_submit
    fails alike, since each checks the whole trace (a rank that succeeded alone
    would wait on its peers in the first exchange)."""
    import numpy as np
    from graphite_amd import gnoc
    from tests.traces import random_trace
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = random_trace(2000, 8, 8, seed=11, max_cycle=3000)
    k = len(tr) // 2
    tr.src[k], tr.dst[k], tr.flags[k] = 5 * 8 + 5, 6 * 8 + 6, 0   # rank 1 of 2: rows 4-7, columns 4-7
    if bad == "zero_flit":
        tr.bits[k] = 0
    elif bad == "too_long":
        tr.bits[k] = 64 * 3000
    else:
        tr.inject_ps[k:] = np.uint64(1 << 50)
    msgs = []
    for r in range(2):
        e = gnoc.Engine(cfg)
        e._check(e.lib.gnoc_shard(e._h, r, 2))
        with pytest.raises(gnoc.GnocError) as ei:
            e.submit(tr)
        msgs.append(str(ei.value))
        e.close()
    assert msgs[0] == msgs[1] and str(k) in msgs[0], msgs


def _rccl_one_rank(cfg, tr, runs=2):
    """gnoc_run_sharded on a 1-rank RCCL communicator of libgnoc's own RCCL."""
    import numpy as np
    from graphite_amd import gnoc
    comm = gnoc.RcclComm(1, 0, 0)
    eng = gnoc.NativeShardedEngine(cfg, 0, 1, comm)
    eng.submit(tr)
    su, ru = np.zeros(1, np.uint64), np.zeros(1, np.uint64)
    eng._check(eng.lib.gnoc_exchange_counts(eng._h, su.ctypes.data, ru.ctypes.data, 1))
    for _ in range(runs):
        eng.run()
    got, summ = eng.results(), eng.summary()
    eng.close()
    comm.close()
    return got, summ, int(su[0]), int(ru[0])


def _unsharded(cfg, tr):
    from graphite_amd import gnoc
    ref = gnoc.Engine(cfg)
    ref.submit(tr)
    ref.run()
    want = ref.results()
    ref.close()
    return want


RESULT_KEYS = ("final_ps", "zero_load_ps", "contention_ps", "port_sum_delay", "port_count", "port_mg1", "port_flit",
               "port_last")


@pytest.mark.parametrize("W,load,ppt", [(8, 0.05, 300), (32, 0.005, 1000)])
def test_rccl_one_rank_self_exchange(W, load, ppt, monkeypatch):
    """gnoc_run_sharded over a real RCCL communicator at one rank, with the
    self-exchange knob: the rank's own turn records (one per routed packet) are
    packed, moved by ncclSend / ncclRecv to itself inside the group, and unpacked
    back into their slots, then the Y phase reads them -- on the stream path (one
    host sync per step, the status all-reduce on the stream).  The results equal
    the unsharded run's and the oracle's."""
    import numpy as np
    from graphite_amd import gnoc
    from oracle import oracle
    monkeypatch.setenv("GNOC_SHARD_SELF_EXCHANGE", "1")
    cfg = gnoc.EngineConfig(num_tiles=W * W)
    tr = gnoc.synthetic_trace(W, W, load, ppt, seed=11)
    got, summ, su, ru = _rccl_one_rank(cfg, tr)
    routed = int(summ["routed_packets"])
    # 16-B units: the pair's status unit, its exception-count header, one record per routed packet
    hdr = 1 + (W * W * 9 + 3) // 4
    assert su == ru == hdr + routed and routed > 0, (su, ru, routed)
    assert summ["fallbacks"] == 0 and summ["engine_path"] == 4, summ
    want = _unsharded(cfg, tr)
    for k in RESULT_KEYS:
        assert np.array_equal(getattr(got, k), getattr(want, k)), k
    if W <= 8:
        orc = oracle.run(cfg, tr)
        assert np.array_equal(got.final_ps, orc.final_ps)


def test_rccl_one_rank_no_self_exchange_is_empty():
    """Without the knob a 1-rank communicator moves nothing (its turn records
    stay in place) and still runs the stream protocol exactly."""
    import numpy as np
    from graphite_amd import gnoc
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, 0.05, 300, seed=12)
    got, summ, su, ru = _rccl_one_rank(cfg, tr)
    assert su == ru == 0
    want = _unsharded(cfg, tr)
    for k in RESULT_KEYS:
        assert np.array_equal(getattr(got, k), getattr(want, k)), k


def test_rccl_declined_x_phase_poisons_and_reruns(monkeypatch):
    """A rank whose X phase does not complete on the stream path (injected once:
    GNOC_DECLINE_ONCE_RANK) marks its send buffer's pair status units; the
    receiving Y phase skips, the step's status all-reduce sends the rank to the
    synchronous protocol, and the rerun is exact.  One fallback is counted."""
    import numpy as np
    from graphite_amd import gnoc
    monkeypatch.setenv("GNOC_SHARD_SELF_EXCHANGE", "1")
    monkeypatch.setenv("GNOC_DECLINE_ONCE_RANK", "0")
    cfg = gnoc.EngineConfig(num_tiles=64)
    tr = gnoc.synthetic_trace(8, 8, 0.05, 300, seed=13)
    comm = gnoc.RcclComm(1, 0, 0)
    eng = gnoc.NativeShardedEngine(cfg, 0, 1, comm)
    eng.submit(tr)
    eng.run()
    s1 = eng.summary()
    first = eng.results()
    for _ in range(3):   # (the windows adapt to the measured fill: an overflow on the next run reruns too)
        eng.run()
    s2 = eng.summary()
    got = eng.results()
    eng.close()
    comm.close()
    assert s1["fallbacks"] >= 1 and s1["runs"] == 1, s1
    assert s2["fallbacks"] == 0 and s2["runs"] == 4, s2
    want = _unsharded(cfg, tr)
    for k in RESULT_KEYS:
        assert np.array_equal(getattr(first, k), getattr(want, k)), k
        assert np.array_equal(getattr(got, k), getattr(want, k)), k
