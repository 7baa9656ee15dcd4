"""The multi-process split grid's host plumbing on CPU (gloo, world_size 2, 127.0.0.1): every
rank arms its part (kss_split_config with its rank), all-gathers the parts' inbox IPC handles in
rank order and opens the same list, also when one rank starts 2 s after the other (the
device-side first exchange then absorbs the skew: tests/test_gpu_split.py::
test_parts_start_apart), and a re-arm after a failed run repeats the whole handshake on every
rank.  The device context is replaced by a recorder: no GPU is touched."""
import os
import socket
import sys
import time

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kube-scheduler-simulator_amd")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Cluster:
    n_nodes = 1000


def _worker(rank, world, port, delay, q):
    sys.path.insert(0, PKG)
    from kss import abi, split

    calls = []

    class Recorder:
        def __init__(self, profile=None, device=0):
            calls.append(("ctx", device))

        def load(self, cluster):
            calls.append(("load", cluster.n_nodes))

        def stage(self, podset):
            calls.append(("stage",))

        def split_config(self, n_parts, part, wl):
            calls.append(("config", n_parts, part, wl))

        def split_inbox(self, with_handle=False):
            calls.append(("inbox",))
            return 0, 0, bytes([0xA0 + rank]) * abi.KSS_IPC_HANDLE_BYTES

        def split_open(self, handles):
            calls.append(("open", [h[0] for h in handles], [len(h) for h in handles]))

        def run_staged(self, n):
            calls.append(("run", n))
            return list(range(n))

        def close(self):
            calls.append(("close",))

    split.native.Context = Recorder
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    time.sleep(delay if rank == 1 else 0.0)  # rank 1's module load / upload takes longer
    t0 = time.time()
    part = split.SplitRank(_Cluster(), None, wl=4, device=0)
    armed = time.time() - t0
    out = part.run(3)
    part.rearm()  # after a failed run: every rank repeats the handshake
    part.close()
    q.put((rank, calls, out, part.rows(), armed))
    dist.barrier()
    dist.destroy_process_group()


def _run(delay):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, delay, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_split_handshake_gloo_world2():
    res = _run(0.0)
    for rank, calls, out, rows, _ in res:
        arm = [("config", 2, rank, 4), ("inbox",), ("open", [0xA0, 0xA1], [64, 64])]
        assert calls == [("ctx", 0), ("load", 1000), ("stage",)] + arm + [("run", 3)] + arm + [("close",)]
        assert out == [0, 1, 2]
    (r0, _, _, rows0, _), (r1, _, _, rows1, _) = res
    assert rows0[1] == rows1[0] and rows0[0] == 0 and rows1[1] == 1000  # the parts tile the rows


def test_split_handshake_tolerates_late_rank():
    """Rank 1 starts 2 s late: rank 0's handshake waits for it (the IPC handles cannot be
    opened before the peer exported them) and both open the same list."""
    res = _run(2.0)
    for rank, calls, _, _, armed in res:
        assert ("open", [0xA0, 0xA1], [64, 64]) in calls
    assert res[0][4] > 1.0  # rank 0 waited for the late rank inside the handshake
