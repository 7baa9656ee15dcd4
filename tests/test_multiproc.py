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
