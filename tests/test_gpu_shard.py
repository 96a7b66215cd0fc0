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
