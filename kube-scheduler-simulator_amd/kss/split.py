"""The node axis as one persistent grid over several GPUs.

Every part loads the whole cluster and stages the same pods; part p runs shards
[p * wl, (p + 1) * wl) of the n_parts * wl shards of k_simple / k_spread and so owns their
node rows.  The per-pod exchanges the kernels already make between their shards
(statistics, PodTopologySpread histograms and critical paths, the packed selectHost key)
become cross-GPU by storing every granule into every part's inbox: xGMI peer stores from
inside the running kernels, polled locally.  A pod costs no kernel launch, no collective
call and no host round trip on any GPU -- the replacement for the per-pod RCCL packed-argmax
all-reduce of kss/nodeaxis.py, which pays two launches and two collectives per pod.

Two drivers:
  InProcessSplit  several parts in one process (one device or several), launched from one
                  thread each so the grids run concurrently (the tests: parts share one GPU);
  SplitRank       one part per process / GPU (torch.distributed carries only the 64-byte
                  IPC handles and the barriers; nothing per pod).

Reference: the per-rank sequence is scheduleOne's findNodesThatPassFilters /
prioritizeNodes / selectHost / AssumePod (simulator/scheduler/scheduler.go:174-219,
232-267, 323-344) over the part's rows.
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import abi, native


def shards_per_part(n_nodes: int, n_parts: int, nodes_per_shard: int = 391, cap: int = 256) -> int:
    """Shards per part so that the whole grid keeps about `nodes_per_shard` nodes per shard
    (the 1-GPU C4 geometry: 100k nodes over 256 shards), at most `cap` per part."""
    total = max(n_parts, -(-max(n_nodes, 1) // nodes_per_shard))
    wl = max(1, min(cap, -(-total // n_parts)))
    # every shard owns at least one node: the grid's n_parts * wl shards never exceed the
    # cluster (the library refuses a split grid it would have to clamp)
    return max(1, min(wl, max(n_nodes, 1) // n_parts))


def part_rows(n_nodes: int, n_parts: int, wl: int, part: int) -> Tuple[int, int]:
    """Canonical rows [lo, hi) a part owns: its shards' row ranges (ceil(N / W) per shard)."""
    W = n_parts * wl
    per = -(-n_nodes // W)
    return min(n_nodes, part * wl * per), min(n_nodes, (part + 1) * wl * per)


def _run_concurrently(fns):
    out: List = [None] * len(fns)
    errs: List = [None] * len(fns)

    def go(i):
        try:
            out[i] = fns[i]()
        except Exception as e:  # noqa: BLE001 - re-raised below
            errs[i] = e

    ts = [threading.Thread(target=go, args=(i,)) for i in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    return out


def _check_co_resident(devices: Sequence[int], wl: int):
    """Every part's grid must be resident at once (the shards poll each other): the parts
    sharing one device need at most one shard per CU between them (a k_spread / k_simple
    shard fills a CU's LDS)."""
    import collections

    import torch
    for dev, k in collections.Counter(devices).items():
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        if k * wl > cus:
            raise ValueError(f"{k} parts x {wl} shards on device {dev} exceed its {cus} CUs: "
                             "the grids could not all be resident")


class InProcessSplit:
    """n_parts contexts in this process, each running its part of one grid."""

    def __init__(self, cluster: abi.Cluster, podset: abi.PodSet, n_parts: int, wl: int,
                 profile: Optional[abi.Profile] = None, devices: Optional[Sequence[int]] = None):
        import gc
        gc.collect()  # contexts no longer referenced release their streams (HIP maps streams onto few HW queues)
        self.n_parts, self.wl, self.n_nodes = n_parts, wl, cluster.n_nodes
        devices = list(devices) if devices is not None else [0] * n_parts
        if len(devices) != n_parts:
            raise ValueError("one device per part")
        _check_co_resident(devices, wl)
        self.ctxs = []
        for p in range(n_parts):
            ctx = native.Context(profile, device=devices[p])
            ctx.load(cluster)
            ctx.stage(podset)
            self.ctxs.append(ctx)
        self.rearm()

    def rearm(self):
        """(Re)configure every part: fresh zeroed inboxes, epochs from 0, peers exchanged.  Needed
        once at the start and after a failed run (the parts' epochs may have drifted apart)."""
        for p, c in enumerate(self.ctxs):
            c.split_config(self.n_parts, p, self.wl)
        inboxes = [c.split_inbox()[0] for c in self.ctxs]
        for c in self.ctxs:
            c.split_peers(inboxes)

    def run(self, n: int) -> List[np.ndarray]:
        """Schedule staged pods [0, n) on every part at once; every part's chosen vector."""
        return _run_concurrently([lambda c=c: c.run_staged(n) for c in self.ctxs])

    def reset(self):
        for c in self.ctxs:
            c.reset()

    def node_state(self):
        """The cluster's mutable columns assembled from the parts' own rows."""
        out = None
        for p, c in enumerate(self.ctxs):
            st = c.node_state()
            lo, hi = part_rows(self.n_nodes, self.n_parts, self.wl, p)
            if out is None:
                out = {k: v.copy() for k, v in st.items()}
            for k in ("requested", "nonzero"):
                out[k][:, lo:hi] = st[k][:, lo:hi]
            out["pod_count"][lo:hi] = st["pod_count"][lo:hi]
            out["class_count"][:, lo:hi] = st["class_count"][:, lo:hi]
            out["term_count"][:, lo:hi] = st["term_count"][:, lo:hi]
        return out

    def close(self):
        for c in self.ctxs:
            c.close()


class SplitRank:
    """This process's part (rank r of world) of a grid over the ranks' GPUs."""

    def __init__(self, cluster: abi.Cluster, podset: abi.PodSet, wl: int, profile: Optional[abi.Profile] = None,
                 device: int = 0, group=None):
        import torch.distributed as dist
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.wl, self.n_nodes = wl, cluster.n_nodes
        self.device = device
        self.ctx = native.Context(profile, device=device)
        self.ctx.load(cluster)
        self.ctx.stage(podset)
        self.rearm()

    def rearm(self):
        """Collective over the group: a fresh inbox and epochs from 0 on every rank, IPC handles
        exchanged.  Once at the start, and on every rank after a failed run on any rank."""
        import torch
        import torch.distributed as dist
        self.ctx.split_config(self.world, self.rank, self.wl)
        _, _, handle = self.ctx.split_inbox(with_handle=True)
        dev = torch.device("cuda", self.device) if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        mine = torch.frombuffer(bytearray(handle), dtype=torch.uint8).to(dev)
        allh = [torch.zeros(abi.KSS_IPC_HANDLE_BYTES, dtype=torch.uint8, device=dev) for _ in range(self.world)]
        dist.all_gather(allh, mine, group=self.group)  # 64 bytes per rank
        self.ctx.split_open([bytes(h.cpu().numpy().tobytes()) for h in allh])
        dist.barrier(group=self.group)

    def run(self, n: int) -> np.ndarray:
        return self.ctx.run_staged(n)

    def rows(self) -> Tuple[int, int]:
        return part_rows(self.n_nodes, self.world, self.wl, self.rank)

    def close(self):
        self.ctx.close()
