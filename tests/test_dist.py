"""The multi-GPU path of bench.py on CPU: world_size 2 over gloo.

Shards are independent (each rank round-trips its own buffer), so the only
collectives are the barrier around the timed region and the MAX / SUM
reductions that turn per-rank times and bytes into the whole-job value.
These tests run bench.py's own helpers with a fake per-rank step whose
duration differs by rank, and check the reported numbers.
"""
import os
import socket
import time

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cpu")
    delay = 0.01 * (rank + 1)  # rank 1 is the slow one
    calls = []

    def step():
        calls.append(1)
        time.sleep(delay)

    elapsed = bench.timed_loop(step, steps=4, warmup=2, world=world, sync=lambda: None, device=dev)
    total = bench.sum_over_ranks(1000.0 * (rank + 1), world, dev)
    q.put((rank, elapsed, total, len(calls)))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bench_collectives_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # every rank sees the same (max) time, bounded below by the slow rank's 4 x 20 ms
    assert res[0][1] == res[1][1]
    assert res[0][1] >= 4 * 0.02
    # whole-job bytes = sum over ranks
    assert res[0][2] == res[1][2] == 3000.0
    # exactly warmup + steps calls per rank
    assert all(r[3] == 6 for r in res)


def test_bench_args_default_to_one_gpu():
    import bench
    a = bench.parse_args([])
    assert a.gpus == 1 and a.steps >= 1 and a.warmup >= 0 and a.config == 2
    assert bench.CONFIGS[2]["gib"] == 4.0 and bench.CONFIGS[2]["dtype"] == "int16"


def test_bench_gpus_spawns_ranks_and_checks_world(monkeypatch):
    """--gpus N outside torch.distributed re-launches bench.py under
    torch.distributed.run with N ranks (as a child process, exiting with its
    status); inside, a world size that differs from --gpus is an error."""
    import bench
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 7)
    with pytest.raises(SystemExit) as ei:
        bench.maybe_spawn(bench.parse_args(["--gpus", "4", "--steps", "3"]), ["--gpus", "4", "--steps", "3"])
    assert ei.value.code == 7
    cmd, env = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "4", "--steps", "3"][-3:]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # one GPU, or already inside torch.distributed: no re-launch
    bench.maybe_spawn(bench.parse_args([]), [])
    monkeypatch.setenv("WORLD_SIZE", "2")
    bench.maybe_spawn(bench.parse_args(["--gpus", "2"]), ["--gpus", "2"])
    assert len(calls) == 1
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit):
        bench.dist_setup(bench.parse_args(["--gpus", "2"]))
