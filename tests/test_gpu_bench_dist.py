"""bench.py's multi-GPU branch on the hardware.

The driver's 8-GPU scaling run goes through bench.py's torch.distributed
path: every rank joins an RCCL ("nccl") process group, and the barrier around
the timed region plus the MAX / SUM all-reduces run on DEVICE tensors.  With
one GPU here, that path is exercised at world size 1: bench.py is started by
torch.distributed.run with --nproc-per-node=1 and --force-dist, which
initialises the RCCL group and runs every collective even for one rank.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_bench_rccl_path_world1():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
           "--gib", "0.25", "--no-cpu-baseline", "--force-dist"]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["dist"] == {"backend": "nccl", "world_size": 1,
                            "collectives": "barrier + all_reduce MAX/SUM on device tensors"}
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["parity"]["round_trip_exact"] is True
