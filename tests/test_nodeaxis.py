"""Node-axis sharding: the row partition, the packed selectHost key and
the two per-pod collectives on CPU (gloo, world_size 2 and 3, 127.0.0.1); on the GPU the
sharded schedule is compared bit-exactly with the C oracle on the whole cluster (chosen
node per pod, per-pod outcome, final node state of every rank's rows)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kss import nodeaxis


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,world", [(100000, 8), (5000, 3), (7, 4), (3, 8), (0, 2), (1, 1)])
def test_row_range_partitions_in_order(n, world):
    ranges = [nodeaxis.row_range(n, r, world) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0 and a0 <= a1
    assert sum(h - l for l, h in ranges) == n


def test_pack_key_orders_like_select_host():
    # higher total wins; on a tie the lower canonical index wins (deterministic tie-break)
    assert nodeaxis.pack_key(5, 10) > nodeaxis.pack_key(4, 0)
    assert nodeaxis.pack_key(5, 10) > nodeaxis.pack_key(5, 11)
    assert nodeaxis.pack_key(0, 99999) > nodeaxis.NO_NODE  # unscored single feasible node still wins
    for total, node in [(0, 0), (900, 99999), (123, 5)]:
        assert nodeaxis.unpack_key(nodeaxis.pack_key(total, node)) == (total, node)
    assert nodeaxis.unpack_key(nodeaxis.NO_NODE) == (0, -1)


def _collective_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(1234)
    n = 1000
    totals = rng.integers(0, 50, n)  # many ties across ranks
    lo, hi = nodeaxis.row_range(n, rank, world)
    local = max((nodeaxis.pack_key(totals[g], g) for g in range(lo, hi)), default=nodeaxis.NO_NODE)
    key = torch.tensor([local], dtype=torch.int64)
    nodeaxis.reduce_key(key)
    stats = torch.tensor([hi - lo, rank * 7, 100 - rank, 0], dtype=torch.int64)
    gathered = torch.zeros(world * nodeaxis.AXIS_STATS, dtype=torch.int64)
    nodeaxis.gather_stats(stats, gathered)
    q.put((rank, int(key.item()), gathered.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_collectives_gloo(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_collective_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(1234)
    totals = rng.integers(0, 50, 1000)
    best = max(range(1000), key=lambda g: (totals[g], -g))
    for rank, key, gathered in out:
        assert nodeaxis.unpack_key(key) == (totals[best], best)
        g = np.array(gathered).reshape(world, nodeaxis.AXIS_STATS)
        assert g[:, 0].sum() == 1000
        assert list(g[:, 1]) == [r * 7 for r in range(world)]


# ---------------------------------------------------------------------------- GPU
def _oracle(config, n_nodes, n_pods):
    import oracle_c
    from kss import abi, native
    s = native.Synth(config, 0, n_nodes, n_pods)
    chosen, res, st = oracle_c.schedule(abi.default_profile(), s.cluster, s.pods, n_pods, n_nodes, record=True,
                                        threads=8)
    meta = np.array([[res.meta(j)[k] for k in ("chosen", "n_feasible", "scored", "status", "best_total")]
                     for j in range(n_pods)], np.int64)
    return chosen, meta, st


def _gpu_worker(rank, world, port, config, n_nodes, n_pods, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kss import abi, native
    s = native.Synth(config, 0, n_nodes, n_pods)
    sch = nodeaxis.NodeAxisScheduler(s.cluster, s.pods, abi.default_profile(), device=0)
    chosen = sch.schedule().cpu().numpy()
    st = sch.node_state()
    q.put((rank, sch.lo, sch.hi, chosen, sch.meta(n_pods), st["requested"], st["pod_count"]))
    dist.barrier()
    sch.close()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("config,n_nodes,n_pods", [(2, 3000, 400), (1, 100, 1000), (1, 3, 50), (5, 1000, 200)])
def test_nodeaxis_world1_matches_oracle(config, n_nodes, n_pods):
    from kss import abi, native
    chosen_o, meta_o, st_o = _oracle(config, n_nodes, n_pods)
    s = native.Synth(config, 0, n_nodes, n_pods)
    sch = nodeaxis.NodeAxisScheduler(s.cluster, s.pods, abi.default_profile(), device=0)
    chosen = sch.schedule().cpu().numpy()
    np.testing.assert_array_equal(chosen, chosen_o)
    np.testing.assert_array_equal(sch.meta(n_pods), meta_o)
    st = sch.node_state()
    np.testing.assert_array_equal(st["requested"][:, :n_nodes], st_o["requested"][:, :n_nodes])
    np.testing.assert_array_equal(st["pod_count"][:n_nodes], st_o["pod_count"][:n_nodes])
    # replay from the snapshot gives the same placements
    sch.reset()
    np.testing.assert_array_equal(sch.schedule().cpu().numpy(), chosen_o)
    sch.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,config,n_nodes,n_pods", [(2, 2, 2000, 300), (3, 2, 1001, 200), (4, 1, 3, 40)])
def test_nodeaxis_gloo_ranks_match_oracle(world, config, n_nodes, n_pods):
    """world ranks share cuda:0 (gloo staging through host tensors), each owning a
    contiguous row block; the union of their results is the whole-cluster oracle's."""
    chosen_o, meta_o, st_o = _oracle(config, n_nodes, n_pods)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, config, n_nodes, n_pods, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=180) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lo, hi, chosen, meta, req, podc in out:
        np.testing.assert_array_equal(chosen, chosen_o, err_msg=f"rank {rank}")
        np.testing.assert_array_equal(meta, meta_o, err_msg=f"rank {rank}")
        np.testing.assert_array_equal(req[:, :hi - lo], st_o["requested"][:, lo:hi], err_msg=f"rank {rank}")
        np.testing.assert_array_equal(podc[:hi - lo], st_o["pod_count"][lo:hi], err_msg=f"rank {rank}")


@pytest.mark.gpu
def test_nodeaxis_custom_profile_matches_oracle():
    """A non-default profile (MostAllocated, changed weights) takes k_axis_eval<false>."""
    import oracle_c
    from kss import abi, native
    prof = abi.default_profile()
    prof.fit_strategy = abi.KSS_FIT_MOST_ALLOCATED
    prof.weight[abi.KSS_S_NODE_AFFINITY] = 5
    prof.weight[abi.KSS_S_BALANCED_ALLOCATION] = 3
    n_nodes, n_pods = 1500, 300
    s = native.Synth(2, 0, n_nodes, n_pods)
    chosen_o, _, st_o = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record=False, threads=8)
    sch = nodeaxis.NodeAxisScheduler(s.cluster, s.pods, prof, device=0)
    np.testing.assert_array_equal(sch.schedule().cpu().numpy(), chosen_o)
    st = sch.node_state()
    np.testing.assert_array_equal(st["requested"][:, :n_nodes], st_o["requested"][:, :n_nodes])
    sch.close()
