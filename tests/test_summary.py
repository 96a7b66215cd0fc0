"""The sim.out network section: send/receive counters,
event counters, contention counters and link utilization, per tile.

CPU: the route-walk event counters of tests/summary_ref.py agree with the
oracle's per-port request counts.  GPU: gnoc_replay --summary all (the C++
plug-in over libgnoc.so) prints exactly the text the reference's formulas give
on the oracle's results."""
import os
import subprocess

import numpy as np
import pytest

from graphite_amd import gnoc
from oracle import oracle
from tests.summary_ref import expected_summary
from tests.traces import random_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "graphite_amd", "_build")


def cases():
    yield "sat8", gnoc.EngineConfig(num_tiles=64), random_trace(6000, 8, 8, seed=3, max_cycle=200, burst0=200,
                                                                   self_frac=0.05, unmodeled_frac=0.05)
    yield "flit16", gnoc.EngineConfig(num_tiles=36, flit_width=16, router_delay=2), random_trace(
        3000, 6, 6, seed=4, max_cycle=900, bits_choices=[72, 576, 1088])
    yield "nocont", gnoc.EngineConfig(num_tiles=16, contention_enabled=False), random_trace(1500, 4, 4, seed=5)
    yield "bcast", gnoc.EngineConfig(num_tiles=20, mesh_width=5, mesh_height=4), random_trace(
        2000, 5, 4, seed=6, max_cycle=2500, self_frac=0.03, unmodeled_frac=0.03, bcast_frac=0.03)


def test_event_counters_match_oracle_requests():
    for _, cfg, tr in cases():
        if not cfg.contention_enabled:
            continue
        ref = oracle.run(cfg, tr)
        for t in range(cfg.width * cfg.height):
            txt = expected_summary(cfg, tr, ref, t)
            # one port per unicast visit: requests = switch allocations, flits = buffer writes
            if not np.any(tr.flags & gnoc.PKT_BROADCAST):
                sar = int(txt.split("Switch Allocator Requests: ")[1].split("\n")[0])
                assert sar == int(ref.port_count[t * 6:t * 6 + 5].sum()), t
                bw = int(txt.split("Buffer Writes: ")[1].split("\n")[0])
                assert bw == int(ref.port_flit[t * 6:t * 6 + 5].sum()), t
            # utilization operands: flits over the router's links (a broadcast visit uses several)
            lt = int(txt.split("Link Traversals: ")[1].split("\n")[0])
            assert lt == int(ref.port_flit[t * 6:t * 6 + 5].sum()), t


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["sat8", "flit16", "nocont", "bcast"])
def test_replay_summary_matches_reference_text(tmp_path, name):
    cfg, tr = next((c, t) for n, c, t in cases() if n == name)
    ref = oracle.run(cfg, tr)
    trace = str(tmp_path / "t.gtr")
    gnoc.write_trace_file(trace, cfg, tr)
    r = subprocess.run([os.path.join(BUILD, "gnoc_replay"), trace, "--summary", "all"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    blocks = r.stdout.split("Tile ")[1:]
    assert len(blocks) == cfg.width * cfg.height
    for b in blocks:
        head, body = b.split(":\n  Network (emesh_hop_by_hop_hip):\n", 1)
        t = int(head)
        body = body.split("{")[0] if t == cfg.width * cfg.height - 1 else body
        assert body == expected_summary(cfg, tr, ref, t), f"tile {t}:\n{body}\nexpected:\n{expected_summary(cfg, tr, ref, t)}"
