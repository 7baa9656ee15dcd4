"""The split grid (kss_split_*, kss/split.py): the node axis as one persistent k_simple /
k_spread grid whose parts run on different GPUs and exchange granules by peer stores.  Here
the parts share the one GPU of the box: in one process (one thread per part) and in two
processes (one part each, inboxes mapped through IPC handles exchanged over gloo).  Every
part's chosen vector and outcomes, and the node state assembled from the parts' own rows,
equal the C oracle's -- on C2's default-profile recipe (k_simple), C4's zone-spread recipe
(k_spread, BASELINE configs[3]) and C3's spread + inter-pod recipe."""
import os

import numpy as np
import pytest

import oracle_c
import split_diag
from kss import abi, native, split
from kss.synth import SEED_BASE

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _oracle(s, n_pods):
    return oracle_c.schedule(abi.default_profile(), s.cluster, s.pods, n_pods, s.n_nodes, record="meta",
                             threads=THREADS, n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)


@pytest.mark.parametrize("config,n_nodes,n_pods,n_parts,wl,kernel", [
    (2, 5000, 600, 2, 8, "k_simple"),
    (4, 20000, 400, 2, 32, "k_spread"),
    (3, 3000, 300, 2, 12, "k_spread"),
    (4, 100000, 200, 2, 128, "k_spread"),
    (4, 100000, 300, 4, 64, "k_spread"),   # BASELINE configs[3] split 4 ways (4 contexts, each on a queue of its own)
    (2, 100000, 300, 4, 32, "k_simple"),
])
def test_in_process_parts_match_oracle(config, n_nodes, n_pods, n_parts, wl, kernel):
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, res, st = _oracle(s, n_pods)
    sp = split.InProcessSplit(s.cluster, s.pods, n_parts, wl)
    for rep in range(2):  # a second run continues the epochs in the inboxes (no clearing)
        sp.reset()
        outs = sp.run(n_pods)
        for p, (c, ch) in enumerate(zip(sp.ctxs, outs)):
            assert c.last_kernel() == kernel
            assert c.last_geometry()["shards"] == n_parts * wl
            np.testing.assert_array_equal(ch, ch_o, err_msg=f"part {p} run {rep}")
    meta = sp.ctxs[-1].fetch_meta(n_pods)
    for j in range(n_pods):
        m = res.meta(j)
        assert (meta[j, 0], meta[j, 1], meta[j, 2], meta[j, 3]) == (m["chosen"], m["n_feasible"], m["scored"],
                                                                    m["status"]), j
    g = sp.node_state()
    N = n_nodes
    np.testing.assert_array_equal(g["requested"][:, :N], st["requested"][:, :N])
    np.testing.assert_array_equal(g["nonzero"][:, :N], st["nonzero"][:, :N])
    np.testing.assert_array_equal(g["pod_count"][:N], st["pod_count"][:N])
    if s.cluster.n_classes:
        np.testing.assert_array_equal(g["class_count"][:s.cluster.n_classes, :N], st["class_count"][:, :N])
    sp.close()


@pytest.mark.parametrize("config,n_nodes,n_pods,per_chunk,wl", [
    (2, 3000, 240, 30, 8),   # k_simple: even chunks (the last and first epochs of adjacent chunks share a parity)
    (2, 3000, 240, 31, 8),
    (4, 6000, 200, 24, 16),  # k_spread: the exchange count per pod is data-dependent
])
def test_parts_over_many_chunks(monkeypatch, config, n_nodes, n_pods, per_chunk, wl):
    """KSS_STATIC_BYTES forces one k_static + one loop launch per `per_chunk` pods: adjacent
    chunks exchange through the two inbox halves, so a part that starts chunk c + 1 never
    overwrites a granule of chunk c that its peer is still polling.  Three runs back to back
    (the chunk sequence continues across runs)."""
    native.set_option("static_bytes", str(4 * n_nodes * per_chunk))
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, res, st = _oracle(s, n_pods)
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)
    N = n_nodes
    nc = s.cluster.n_classes
    init_cc = np.ctypeslib.as_array(s.cluster.class_count, shape=(max(nc, 1) * N,)).reshape(max(nc, 1), N)[:nc]
    for rep in range(3):
        sp.reset()
        try:
            outs = sp.run(n_pods)
        except native.KssError:
            _handoff_report(sp, rep, failed=True)
            raise
        bad = [np.flatnonzero(np.asarray(ch) != ch_o) for ch in outs]
        g = sp.node_state()
        if any(len(b) for b in bad) or (s.cluster.n_classes and not np.array_equal(
                g["class_count"][:s.cluster.n_classes, :N], st["class_count"][:, :N])):
            split_diag.report(sp, s.pods, init_cc, n_pods, wl, per_chunk, split.part_rows)  # trace builds only
        if any(len(b) for b in bad):  # what went wrong, for the record: pod, chunk position, outcomes
            j = int(next(b for b in bad if len(b))[0])
            meta = [c.fetch_meta(n_pods)[j].tolist() for c in sp.ctxs]
            m = res.meta(j)
            pytest.fail(f"run {rep}: mismatching pods per part {[b.tolist() for b in bad]}; first {j} = chunk "
                        f"{j // per_chunk} pod {j % per_chunk}; device {[o[j] for o in outs]} meta {meta}; oracle "
                        f"{ch_o[j]} meta {[m['chosen'], m['n_feasible'], m['scored'], m['status'], m['best_total']]}")
        assert sp.ctxs[0].last_timing()[1] == 2 * -(-n_pods // per_chunk)  # k_static + loop per chunk
        # the node state every run leaves, count rows included (a wrong count need not change a choice)
        np.testing.assert_array_equal(g["requested"][:, :N], st["requested"][:, :N], err_msg=f"run {rep}")
        np.testing.assert_array_equal(g["pod_count"][:N], st["pod_count"][:N], err_msg=f"run {rep}")
        for key, n_rows in (("class_count", s.cluster.n_classes), ("term_count", s.cluster.n_terms)):
            if n_rows:
                d = np.argwhere(g[key][:n_rows, :N] != st[key][:n_rows, :N])
                assert not len(d), (f"run {rep}: {key} differs at (row, node, device, oracle) " + str(
                    [(int(a), int(b), int(g[key][a, b]), int(st[key][a, b])) for a, b in d[:8]]))
        _handoff_report(sp, rep)
    sp.close()


def _handoff_report(sp, rep, failed=False):
    """The node-state hand-off check of every part after a run (k_spread chunks): reloads, loads
    the shadow copy answered, and the words where state and shadow differed.  Printed when any
    reload happened, and appended to $KSS_HANDOFF_LOG when set (evidence for DESIGN §5)."""
    lines = []
    for p, c in enumerate(sp.ctxs):
        retries = c.last_handoff_retries()
        if not retries:
            continue
        rec, entries = c.last_handoff_diag()
        lines.append(f"run {rep} part {p}{' FAILED' if failed else ''}: reloads {retries}, shadow answered {rec}, "
                     f"differing words {len(entries)}")
        lines += [f"  {e}" for e in entries[:16]]
        for e in entries[:4]:  # which buffer of which part holds the word, and its neighbours
            for q, c2 in enumerate(sp.ctxs):
                for nm, (b, sz) in c2.buffer_map().items():
                    if b and b - (1 << 22) <= e["addr"] < b + sz + (1 << 22):
                        lines.append(f"    word {e['addr']:#x}: part {q} {nm} [{b:#x}, +{sz}) offset {e['addr'] - b}")
    if lines:
        allb = sorted((b, sz, q, nm) for q, c2 in enumerate(sp.ctxs) for nm, (b, sz) in c2.buffer_map().items() if b)
        lines.append("  buffers: " + ", ".join(f"p{q}.{nm}@{b:#x}+{sz}" for b, sz, q, nm in allb))
        print("\n".join(lines))
        if os.environ.get("KSS_HANDOFF_LOG"):
            with open(os.environ["KSS_HANDOFF_LOG"], "a") as f:
                f.write("\n".join(lines) + "\n")
    for p, c in enumerate(sp.ctxs):  # a repaired hand-off is a failure, not a footnote
        assert c.last_handoff_status() == {"reloads": 0, "shadow": 0, "final": 0}, (p, "\n".join(lines))


def test_shards_per_part_never_exceed_nodes():
    assert split.shards_per_part(1, 2) == 1 and split.shards_per_part(3, 2) == 1
    assert split.shards_per_part(100000, 8) == 32
    s = native.Synth(2, SEED_BASE + 2, 6, 4)
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    ctx.split_config(2, 0, 4)  # 8 shards over 6 nodes
    ctx.split_peers([ctx.split_inbox()[0]] * 2)
    with pytest.raises(native.KssError, match="more shards than nodes"):
        ctx.run_staged(4)
    ctx.close()


def _n_devices():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_n_devices() < 2, reason="needs 2 GPUs (the xGMI peer stores of a split grid)")
@pytest.mark.parametrize("config,n_nodes,n_pods,wl", [(2, 5000, 400, 8), (4, 100000, 200, 128)])
def test_two_devices_in_process(config, n_nodes, n_pods, wl):
    """The split grid's deployment shape: parts on different GPUs, every granule stored into
    the peer's inbox over xGMI."""
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, _, st = _oracle(s, n_pods)
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl, devices=[0, 1])
    for rep in range(2):
        sp.reset()
        for p, ch in enumerate(sp.run(n_pods)):
            np.testing.assert_array_equal(ch, ch_o, err_msg=f"part {p} run {rep}")
    g = sp.node_state()
    np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    sp.close()


def test_split_refuses_what_it_cannot_run():
    s = native.Synth(2, SEED_BASE + 2, 500, 50)
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    ctx.split_config(2, 0, 4)
    with pytest.raises(native.KssError):  # peers not set
        ctx.run_staged(10)
    with pytest.raises(native.KssError):  # recorded batches stay on k_schedule
        ctx.schedule_batch(s.pods, 10, record=True)
    ctx.split_config(1, 0, 1)  # back to the whole grid on this device
    ch_o, _, _ = _oracle(s, 50)
    np.testing.assert_array_equal(ctx.run_staged(50), ch_o)
    ctx.close()


def test_failed_run_refuses_until_rearmed():
    """A part whose peer never runs times out in its first exchange; its epochs are then
    apart from the peer's, so it refuses split runs until every part is re-armed."""
    s = native.Synth(2, SEED_BASE + 2, 2000, 40)
    ch_o, _, _ = _oracle(s, 40)
    sp = split.InProcessSplit(s.cluster, s.pods, 2, 4)
    with pytest.raises(native.KssError):  # part 1 never runs: part 0's exchange times out
        sp.ctxs[0].run_staged(40)
    with pytest.raises(native.KssError, match="re-arm"):
        sp.ctxs[0].run_staged(40)
    sp.rearm()
    sp.reset()
    for p, ch in enumerate(sp.run(40)):
        np.testing.assert_array_equal(ch, ch_o, err_msg=f"part {p}")
    sp.close()


def test_parts_start_apart():
    """Part 1 launches its grid 2 s after part 0 (a peer process that starts late: module
    load, IPC open): part 0's first exchange waits for it -- every exchange wait is bounded
    by wall time (10 s), not by a poll count -- and both parts equal the oracle, twice."""
    import time
    config, n_nodes, n_pods, wl = 4, 20000, 300, 32
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, _, _ = _oracle(s, n_pods)
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)

    def late(c):
        time.sleep(2.0)
        return c.run_staged(n_pods)

    for rep, (a, b) in enumerate([(0, 1), (1, 0)]):  # each part once the late one
        sp.reset()
        outs = split._run_concurrently([lambda: sp.ctxs[a].run_staged(n_pods), lambda: late(sp.ctxs[b])])
        for p, ch in zip((a, b), outs):
            np.testing.assert_array_equal(ch, ch_o, err_msg=f"part {p} (late part {b})")
    sp.close()


def _rank_main(rank, world, port, config, n_nodes, n_pods, wl, q, device_of=None):
    import torch
    import torch.distributed as dist
    try:
        dev = device_of(rank) if device_of else 0
        torch.cuda.set_device(dev)
        torch.zeros(1, device="cuda")  # torch's HIP runtime before libkss's
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
        r = split.SplitRank(s.cluster, s.pods, wl, device=dev)
        chosen = r.run(n_pods)
        lo, hi = r.rows()
        st = r.ctx.node_state()
        q.put((rank, chosen.tolist(), lo, hi, st["requested"][:, lo:hi].tolist(), r.ctx.last_kernel(),
               r.ctx.last_handoff_status()))
        dist.barrier()
        r.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e), 0, 0, None, None, None))


def _identity(r):
    return r


@pytest.mark.parametrize("world,config,n_nodes,n_pods,wl,two_gpus", [
    (2, 4, 20000, 300, 32, False),
    pytest.param(2, 4, 20000, 300, 32, True, marks=pytest.mark.skipif(_n_devices() < 2, reason="needs 2 GPUs")),
    # the 8-GPU node's shape, rehearsed on one GPU: 8 processes, 32 shards each (C4: 100k nodes),
    # every granule published into 8 inboxes
    (8, 4, 100000, 200, 32, False),
])
def test_processes_through_ipc_handles(world, config, n_nodes, n_pods, wl, two_gpus):
    """One part per process (the deployment shape: one process per GPU), inboxes mapped
    through hipIpcOpenMemHandle, the handles exchanged over gloo; every process's grid on
    the box's one GPU at once, or (two_gpus) rank r on GPU r, peer stores over xGMI."""
    import multiprocessing as mp
    import socket
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, _, st = _oracle(s, n_pods)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, config, n_nodes, n_pods, wl, q,
                                               _identity if two_gpus else None)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, chosen, lo, hi, req, kernel, handoff in got:
        assert req is not None, chosen  # the child's exception
        assert kernel == "k_spread"
        assert handoff == {"reloads": 0, "shadow": 0, "final": 0}, (rank, handoff)
        np.testing.assert_array_equal(np.array(chosen), ch_o, err_msg=f"rank {rank}")
        np.testing.assert_array_equal(np.array(req, dtype=np.int64).reshape(abi.KSS_NRES, hi - lo),
                                      st["requested"][:, lo:hi], err_msg=f"rank {rank}")


def _few_queues_main(queues, config, n_nodes, n_pods, n_parts, wl, q):
    os.environ["GPU_MAX_HW_QUEUES"] = str(queues)  # before this child's HIP runtimes start
    try:
        import torch
        torch.zeros(1, device="cuda")
        s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
        sp = split.InProcessSplit(s.cluster, s.pods, n_parts, wl)
        outs = []
        for _ in range(2):
            sp.reset()
            outs.append([ch.tolist() for ch in sp.run(n_pods)])
        st = [c.last_handoff_status() for c in sp.ctxs]
        sp.close()
        q.put((outs, st, None))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((None, None, repr(e)))


@pytest.mark.parametrize("queues", [1, 4])
def test_parts_on_few_hardware_queues(queues):
    """The r5d failure's configuration: 4 in-process parts at or below the runtime's
    hardware-queue count (4 is the box's default; 1 shares every plain stream).  Plain streams
    on a shared queue run their kernels one after the other, so the parts would wait out the
    exchange bound; kss_split_config gives each part a queue of its own, and every part equals
    the oracle, twice, with clean hand-offs."""
    import multiprocessing as mp
    config, n_nodes, n_pods, n_parts, wl = 4, 20000, 200, 4, 16
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, _, _ = _oracle(s, n_pods)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_few_queues_main, args=(queues, config, n_nodes, n_pods, n_parts, wl, q))
    p.start()
    outs, st, err = q.get(timeout=100)
    p.join(timeout=30)
    assert err is None, err
    for rep, run in enumerate(outs):
        for part, ch in enumerate(run):
            np.testing.assert_array_equal(np.array(ch), ch_o, err_msg=f"part {part} run {rep}")
    assert all(x == {"reloads": 0, "shadow": 0, "final": 0} for x in st), st
