"""Multi-GPU control plane on CPU (gloo, world_size 2, 127.0.0.1): the scenario-sharded
bench reduces timing with MAX and work with SUM over ranks, and every rank schedules
a distinct independent cluster (rank 0 = the canonical BASELINE cluster)."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed, total = bench.reduce_over_ranks(1.0 + rank, 100 * (rank + 1), dist)
    q.put((rank, elapsed, total))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_over_ranks_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, elapsed, total in out:
        assert elapsed == 2.0  # slowest rank
        assert total == 300    # all ranks' pods


def test_single_process_reduction_is_identity():
    assert bench.reduce_over_ranks(1.5, 7, None) == (1.5, 7)


@pytest.mark.parametrize("cfg", [1, 2, 5])
def test_rank_seeds_distinct_and_rank0_canonical(cfg):
    from kss.synth import SEED_BASE
    seeds = [bench.rank_seed(SEED_BASE, cfg, r) for r in range(8)]
    assert seeds[0] == SEED_BASE + cfg
    assert len(set(seeds)) == 8


def test_gpus_beyond_visible_fail_clearly(monkeypatch, capsys):
    monkeypatch.setattr(bench, "visible_gpus", lambda: 1)
    assert bench.launch_ranks(2, ["--gpus", "2"]) == 2
    assert "2 GPUs requested, 1 visible" in capsys.readouterr().err


def test_launcher_starts_one_rank_per_gpu(monkeypatch):
    """Without torchrun, `--gpus N` starts torch.distributed.run with N ranks on 127.0.0.1
    and returns its exit code (this process never opens the GPU)."""
    seen = {}
    monkeypatch.setattr(bench, "visible_gpus", lambda: 8)
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, cwd=None: seen.setdefault("cmd", cmd) and 0)
    assert bench.launch_ranks(4, ["--gpus", "4", "--steps", "2"]) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]


def _leg_worker(rank, world, port, fail_rank, q):
    import argparse
    import subprocess
    import types
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = {}

    def fake_run(cmd, cwd=None, env=None, capture_output=None, text=None, timeout=None):
        seen["env"] = env
        rc = 1 if rank == fail_rank else 0
        out = '{"value": 5.0, "n_gpus": %d}\n' % world if rank == 0 else ""
        return types.SimpleNamespace(returncode=rc, stdout=out, stderr="boom" if rc else "")

    subprocess.run = fake_run
    args = argparse.Namespace(steps=2, warmup=1, cpu_seconds=12.0, no_cpu=True, c4_timeout=10.0)
    res = bench.c4_split_leg(args, world, rank, rank, dist)
    env = seen["env"]
    q.put((rank, res, env["RANK"], env["WORLD_SIZE"], env["LOCAL_RANK"], env["MASTER_PORT"]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_c4_split_leg_gloo_world2(fail_rank):
    """The C4 split leg's control plane: rank 0's port reaches every rank's child environment,
    rank 0 returns its child's line, and a failing peer child turns into an error field."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_leg_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ports = {o[5] for o in out}
    assert len(ports) == 1 and ports != {str(port)}
    assert [(o[2], o[3], o[4]) for o in out] == [("0", "2", "0"), ("1", "2", "1")]
    res0 = out[0][1]
    assert res0["n_gpus"] == 2 and res0["value"] == 5.0
    if fail_rank == 1:
        assert "error" in res0
    else:
        assert "error" not in res0
    assert out[1][1] == {}
