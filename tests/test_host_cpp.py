"""The C++ host side (graphite_amd/host: the NetworkModel-shaped plug-in over
the C ABI) and the on-disk trace format.

CPU: trace files round-trip.  GPU: the C++ known-answer test binary, and every
committed golden trace replayed by gnoc_replay through the C++ model, compared
bit-exactly with the golden outputs (which the CPU oracle produced)."""
import json
import os
import subprocess

import numpy as np
import pytest

from graphite_amd import gnoc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "graphite_amd", "_build")
GOLD = os.path.join(ROOT, "tests", "golden")
GOLDEN = sorted(f[:-4] for f in os.listdir(GOLD) if f.endswith(".npz"))


def _golden(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    cfg = gnoc.EngineConfig(**json.loads(str(z["cfg"])))
    return cfg, gnoc.Trace(z["inject_ps"], z["src"], z["dst"], z["bits"], z["flags"]), z


def test_trace_file_round_trip(tmp_path):
    cfg, tr, _ = _golden("g_6x6_flit16_r2")
    p = str(tmp_path / "t.gtr")
    gnoc.write_trace_file(p, cfg, tr)
    cfg2, tr2 = gnoc.read_trace_file(p)
    assert (cfg2.num_tiles, cfg2.flit_width, cfg2.router_delay) == (36, 16, 2)
    for k in ("inject_ps", "src", "dst", "bits", "flags"):
        assert np.array_equal(getattr(tr2, k), getattr(tr.normalized(), k)), k


def test_trace_file_rejects_garbage(tmp_path):
    p = tmp_path / "bad.gtr"
    p.write_bytes(b"not a trace" * 20)
    with pytest.raises(gnoc.GnocError):
        gnoc.read_trace_file(str(p))


def test_trace_header_carries_moving_average(tmp_path):
    """Header v2 round trip of the basic queue's moving average; a version-1 file
    (no such keys) reads with none, as the reference's defaults give."""
    cfg = gnoc.EngineConfig(num_tiles=16, queue_type=gnoc.QUEUE_BASIC,
                            moving_avg_type=gnoc.MOVING_AVG_MEDIAN, moving_avg_window=17)
    tr = gnoc.Trace(np.array([0, 5, 9], np.uint64), np.array([0, 1, 2], np.uint32), np.array([3, 2, 1], np.uint32),
                    np.array([576, 576, 72], np.uint32))
    p = str(tmp_path / "q.gtr")
    gnoc.write_trace_file(p, cfg, tr)
    c2, t2 = gnoc.read_trace_file(p)
    assert (c2.moving_avg_type, c2.moving_avg_window) == (gnoc.MOVING_AVG_MEDIAN, 17)
    assert np.array_equal(t2.inject_ps, tr.inject_ps) and np.array_equal(t2.bits, tr.bits)
    raw = bytearray(open(p, "rb").read())
    assert int.from_bytes(raw[8:12], "little") == 2
    raw[8:12] = (1).to_bytes(4, "little")
    p1 = str(tmp_path / "v1.gtr")
    open(p1, "wb").write(bytes(raw))
    c1, _ = gnoc.read_trace_file(p1)
    assert c1.moving_avg_type == gnoc.MOVING_AVG_NONE


@pytest.mark.gpu
def test_cpp_sharded_run_through_c_transport():
    """gnoc_run_sharded over the in-process C transport (2, 3, 5 ranks == unsharded;
    a failure on one rank fails all): multi-GPU without Python or torch."""
    r = subprocess.run([os.path.join(BUILD, "test_shard_transport")], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "every rank failed" in r.stdout


@pytest.mark.gpu
def test_replay_sharded_matches_unsharded(tmp_path):
    """gnoc_replay --shards 4 (C ABI, in-process transport) writes the same results
    file as the unsharded replay."""
    cfg = gnoc.EngineConfig(num_tiles=256)
    tr = gnoc.synthetic_trace(16, 16, 0.01, 200, seed=4)
    trace = str(tmp_path / "t.gtr")
    gnoc.write_trace_file(trace, cfg, tr)
    outs = []
    for extra in ([], ["--shards", "4"]):
        out = str(tmp_path / f"r{len(outs)}.bin")
        r = subprocess.run([os.path.join(BUILD, "gnoc_replay"), trace, "--results", out] + extra, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stderr
        outs.append(np.fromfile(out, np.uint64))
    assert outs[0].size == outs[1].size and np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
def test_cpp_known_answers():
    r = subprocess.run([os.path.join(BUILD, "test_emesh_hop_by_hop_hip")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name", GOLDEN)
def test_replay_golden_through_cpp_model(tmp_path, name):
    cfg, tr, z = _golden(name)
    trace = str(tmp_path / "t.gtr")
    out = str(tmp_path / "r.bin")
    gnoc.write_trace_file(trace, cfg, tr)
    # the header (v2) carries the basic queue's moving average: no command-line flag
    r = subprocess.run([os.path.join(BUILD, "gnoc_replay"), trace, "--results", out, "--summary", "0"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Total Packets Received" in r.stdout
    n, np_ = len(tr), cfg.width * cfg.height * gnoc.PORTS_PER_TILE
    a = np.fromfile(out, np.uint64)
    assert a.size == 3 * n + 3 * np_
    got = dict(final_ps=a[:n], zero_load_ps=a[n:2 * n], contention_ps=a[2 * n:3 * n],
               port_sum_delay=a[3 * n:3 * n + np_], port_count=a[3 * n + np_:3 * n + 2 * np_],
               port_mg1=a[3 * n + 2 * np_:])
    for k, v in got.items():
        assert np.array_equal(v, z[k]), k
