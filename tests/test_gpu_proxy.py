"""The 1024-tile proxy app trace (tests/golden/make_proxy.py: MSI shared-memory
lengths 72 b / 584 b, ACKwise-style invalidation broadcasts) against the oracle's
SHA-256 pins, through the Python engine and through the C++ model's trace
replay (gnoc_replay), every result array bit-exact."""
import json
import os
import subprocess

import numpy as np
import pytest

from graphite_amd import gnoc
from tests.golden.make_proxy import RESULT_FIELDS, proxy_trace, sha, trace_hash

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "proxy_hashes.json")) as _fh:
    GOLD = json.load(_fh)
BUILD = os.path.join(os.path.dirname(HERE), "graphite_amd", "_build")


def _trace():
    tr = proxy_trace()
    assert trace_hash(tr) == GOLD["trace_sha256"], "proxy trace generator changed"
    return tr


def test_proxy_trace_engine_matches_oracle():
    tr = _trace()
    eng = gnoc.Engine(gnoc.EngineConfig(num_tiles=1024))
    eng.submit(tr)
    eng.run()
    res = eng.results()
    eng.close()
    bad = [f for f in RESULT_FIELDS if sha(getattr(res, f)) != GOLD["results"][f]["sha256"]]
    assert not bad, {f: (int(getattr(res, f).astype(np.uint64).sum(dtype=np.uint64)), GOLD["results"][f]["sum"])
                     for f in bad}


def test_proxy_trace_replay_through_cpp_model(tmp_path):
    tr = _trace()
    trace, out = str(tmp_path / "proxy.gtr"), str(tmp_path / "r.bin")
    gnoc.write_trace_file(trace, gnoc.EngineConfig(num_tiles=1024), tr)
    r = subprocess.run([os.path.join(BUILD, "gnoc_replay"), trace, "--results", out], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    n, np_ = len(tr), 1024 * gnoc.PORTS_PER_TILE
    a = np.fromfile(out, np.uint64)
    assert a.size == 3 * n + 3 * np_
    got = dict(final_ps=a[:n], zero_load_ps=a[n:2 * n], contention_ps=a[2 * n:3 * n],
               port_sum_delay=a[3 * n:3 * n + np_], port_count=a[3 * n + np_:3 * n + 2 * np_], port_mg1=a[3 * n + 2 * np_:])
    for f, v in got.items():
        assert sha(v) == GOLD["results"][f]["sha256"], f
