"""Node-axis sharding of one cluster over several GPUs.

Every rank owns a contiguous canonical row range of the cluster and stages the same
pending pods.  A pod is scheduled with two HIP launches per rank and two small
collectives between them, all enqueued on one stream of the rank, so the host never
waits on the device inside the pod loop:

    kss_axis_eval     the previous pod's pending AssumePod (owning rank), then filter
                      chain + raw scores of the local rows, local statistics
    all_gather        {feasible count, max TaintToleration raw, max NodeAffinity raw}
    kss_axis_select   NormalizeScore with the global statistics, weighted total, local
                      packed selectHost key (total << 32 | 0xFFFFFFFF - global index)
    all_reduce MAX    the packed key: the winner and the lowest-index tie-break at once

and kss_axis_commit applies the last pod's AssumePod.  The statistics and key buffers
are double-buffered by pod parity (include/kss.h).

Under the ``nccl`` backend (RCCL over xGMI) the collectives run on device tensors;
under ``gloo`` (CPU tests, several ranks sharing one GPU) the 32-byte statistics and the
8-byte key are staged through host tensors.  Both messages are a few dozen bytes, so the
node-axis mode is latency-bound per pod (two collective round trips), not
bandwidth-bound, and is reported that way.

Reference: the sequence replaced per rank is scheduleOne's findNodesThatPassFilters /
prioritizeNodes / selectHost / AssumePod (the
simulator's mirror is simulator/scheduler/scheduler.go:174-219, 232-267, 323-344).
"""
from __future__ import annotations

from typing import Optional, Tuple

from . import abi, native

AXIS_STATS = 4   # int64 per fold slot (KSS_AXIS_STATS)
AXIS_SLOTS = 32  # fold slots per rank (KSS_AXIS_SLOTS): stats [SLOTS][STATS], key [SLOTS]
NO_NODE = 0     # packed key of "no feasible node"


def row_range(n_nodes: int, rank: int, world: int) -> Tuple[int, int]:
    """Canonical rows [lo, hi) owned by `rank`: contiguous blocks of ceil(N / world)."""
    per = -(-n_nodes // world) if world > 0 else n_nodes
    lo = min(n_nodes, rank * per)
    return lo, min(n_nodes, lo + per)


def pack_key(total: int, node: int) -> int:
    """selectHost key of kss_axis.cuh: higher total wins, then the lower canonical index."""
    return (int(total) << 32) | (0xFFFFFFFF - int(node))


def unpack_key(key: int) -> Tuple[int, int]:
    """(total, node) of a packed key; node -1 for NO_NODE."""
    if key == NO_NODE:
        return 0, -1
    return key >> 32, 0xFFFFFFFF - (key & 0xFFFFFFFF)


def gather_stats(stats, gathered, group=None):
    """all_gather of the per-rank statistics vector into gathered[world * len(stats)]."""
    import torch
    import torch.distributed as dist
    if stats.device.type == "cpu" or dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(gathered, stats, group=group)
        return
    host = stats.cpu()
    out = torch.empty(gathered.numel(), dtype=stats.dtype)
    dist.all_gather_into_tensor(out, host, group=group)
    gathered.copy_(out)


def reduce_key(key, group=None):
    """Elementwise all_reduce MAX of the packed selectHost key slots (non-negative int64)."""
    import torch.distributed as dist
    if key.device.type == "cpu" or dist.get_backend(group) != "gloo":
        dist.all_reduce(key, op=dist.ReduceOp.MAX, group=group)
        return
    host = key.cpu()
    dist.all_reduce(host, op=dist.ReduceOp.MAX, group=group)
    key.copy_(host)


class NodeAxisScheduler:
    """One rank's share of a node-axis sharded cluster on one GPU."""

    def __init__(self, cluster: abi.Cluster, podset: abi.PodSet, profile: Optional[abi.Profile] = None,
                 device: int = 0, group=None):
        import torch
        import torch.distributed as dist
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1
        self.n_nodes = cluster.n_nodes
        self.n_pods = podset.n_pods
        self.lo, self.hi = row_range(cluster.n_nodes, self.rank, self.world)
        self.device = torch.device("cuda", device)
        # torch's bundled HIP runtime must open the device before libkss.so's /opt/rocm runtime
        # does (the other order leaves torch with "No HIP GPUs are available")
        torch.zeros(1, device=self.device)
        self.ctx = native.Context(profile, device=device)
        self.ctx.load_rows(cluster, self.lo, self.hi)
        self.ctx.stage(podset)
        i64 = torch.int64
        self.stats = torch.zeros(2, AXIS_SLOTS * AXIS_STATS, dtype=i64, device=self.device)  # [pod parity]
        self.gathered = None if self.world == 1 else torch.zeros(self.world * AXIS_SLOTS * AXIS_STATS, dtype=i64,
                                                                 device=self.device)
        self.key = torch.zeros(2, AXIS_SLOTS, dtype=i64, device=self.device)
        self.chosen = torch.full((max(self.n_pods, 1),), -2, dtype=torch.int32, device=self.device)
        # a stream of our own: torch's default stream has handle 0, which the C ABI reads as
        # "the context's stream" and would not be ordered with the collectives
        self.stream = torch.cuda.Stream(device=self.device)

    def reset(self):
        """Restore the snapshot's node state (every rank) for a replay."""
        self.stream.synchronize()
        self.ctx.reset()
        self.stats.zero_()
        self.key.zero_()

    def schedule(self, n: Optional[int] = None):
        """Schedule pods [0, n) sequentially; returns the device tensor of chosen global nodes."""
        import torch
        n = self.n_pods if n is None else n
        if n > self.n_pods:
            raise ValueError("n exceeds the staged pods")
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        ctx, W = self.ctx, self.world
        sp = [self.stats[b].data_ptr() for b in (0, 1)]
        kp = [self.key[b].data_ptr() for b in (0, 1)]
        cp = self.chosen.data_ptr()
        gp = [self.gathered.data_ptr()] * 2 if W > 1 else sp  # world 1: the statistics are global
        with torch.cuda.stream(self.stream):
            stream = self.stream.cuda_stream
            for i in range(n):
                b = i & 1
                ctx.axis_eval(i, sp[b], kp[1 - b] if i else 0, gp[1 - b] if i else 0, W, kp[b], cp, stream)
                if W > 1:
                    gather_stats(self.stats[b], self.gathered, self.group)
                ctx.axis_select(gp[b], W, kp[b], sp[1 - b], stream)
                if W > 1:
                    reduce_key(self.key[b], self.group)
            if n:
                ctx.axis_commit(n - 1, kp[(n - 1) & 1], gp[(n - 1) & 1], W, cp, stream)
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        return self.chosen[:n]

    def meta(self, n: int):
        """(n, 5) int64 per-pod outcome (chosen, n_feasible, scored, status, best_total)."""
        return self.ctx.fetch_meta(n)

    def node_state(self):
        self.stream.synchronize()
        return self.ctx.node_state()

    def close(self):
        self.ctx.close()
