"""percentageOfNodesToScore below 100 on the device: numFeasibleNodesToFind and
nextStartNodeIndex (v1.26 findNodesThatPassFilters, Parallelism = 1) on k_schedule, against the
C oracle -- chosen nodes, per-pod outcomes, every per-node record (the unvisited nodes, the node
that ended the search, scores over the kept nodes), the final node state and the cursor --
through every entry point that runs a scheduling cycle: recorded and unrecorded batches (one
and several workgroups), staged runs continued across launches, the per-pod API, the service
grid and scenario sweeps.  Staged default-profile batches run the window on k_simple
(simple_sync_win: per-wave and per-thread modes, one and several shards, XCD-local or not,
several chunk launches handing the cursor on); k_spread refuses it (tests/test_plan.py)."""
import os

import numpy as np
import pytest

import oracle_c
from kss import abi, native
from kss.compile import compile_cluster
from kss.synth import SEED_BASE

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _prof(pct):
    p = abi.default_profile()
    p.pct_nodes_to_score = pct
    return p


def _oracle(prof, cl, ps, n, N, record=True, n_classes=0, n_terms=0, cursor=0):
    return oracle_c.schedule(prof, cl, ps, n, N, record=record, threads=THREADS, n_classes=n_classes,
                             n_terms=n_terms, cursor=cursor)


def _meta_equal(meta, res, n):
    for j in range(n):
        m = res.meta(j)
        got = dict(chosen=meta[j, 0], n_feasible=meta[j, 1], scored=meta[j, 2], status=meta[j, 3])
        assert got == {k: m[k] for k in got}, (j, got, m)
        if m["scored"]:
            assert meta[j, 4] == m["best_total"], j


def _record_equal(r, res, j, N):
    """One pod's device record against the oracle's: verdicts and details on every node, scores
    on the kept nodes (feasible and not the dropped one)."""
    np.testing.assert_array_equal(r.fail_plugin[:N], res.fail_plugin[j, :N], err_msg=f"pod {j} verdicts")
    np.testing.assert_array_equal(r.fail_detail[:N], res.fail_detail[j, :N], err_msg=f"pod {j} details")
    m = res.meta(j)
    assert (r.chosen, r.n_feasible, r.scored, r.status) == (m["chosen"], m["n_feasible"], m["scored"], m["status"]), j
    if m["scored"]:
        kept = (res.fail_plugin[j, :N] == 0) & (res.fail_detail[j, :N] != abi.KSS_PASS_NOT_KEPT)
        np.testing.assert_array_equal(r.raw[:, :N][:, kept], res.raw[j][:, :N][:, kept], err_msg=f"pod {j} raw")
        np.testing.assert_array_equal(r.norm[:, :N][:, kept], res.norm[j][:, :N][:, kept], err_msg=f"pod {j} norm")
        np.testing.assert_array_equal(r.total[:N][kept], res.total[j, :N][kept], err_msg=f"pod {j} total")


@pytest.mark.parametrize("pct", [0, 30])
@pytest.mark.parametrize("flags", [0, abi.KSS_SCHED_FORCE_SINGLE_WG])
def test_c2_window_records(pct, flags):
    """BASELINE configs[1]'s cluster (5,000 nodes: K = 500 adaptive, 1,500 at 30 %), 400 pods
    with every per-node record, on the sharded grid (the per-shard count exchange) and on one
    workgroup."""
    n_nodes, n_pods = 5000, 400
    prof = _prof(pct)
    s = native.Synth(2, SEED_BASE + 2, n_nodes, n_pods)
    ch_o, res, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes)
    ctx = native.Context(prof, max_pods_record=n_pods)
    ctx.load(s.cluster)
    chosen = ctx.schedule_batch(s.pods, n_pods, record=True, flags=flags)
    assert ctx.last_kernel() == "k_schedule"
    if not flags:
        assert ctx.last_geometry()["shards"] > 1
    np.testing.assert_array_equal(chosen, ch_o)
    dropped = 0
    for j in range(n_pods):
        r = ctx.fetch_record(j)
        _record_equal(r, res, j, n_nodes)
        dropped += int((r.fail_detail[:n_nodes] == abi.KSS_PASS_NOT_KEPT).sum())
    assert dropped > n_pods // 2  # the search stopped early for most pods
    assert ctx.next_start_node_index() == st["next_start"]
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    ctx.close()


@pytest.mark.parametrize("kernel", ["k_simple", "k_schedule"])
@pytest.mark.parametrize("pct", [0, 30])
def test_c2_full_batch_window(pct, kernel):
    """The whole C2 batch (5,000 nodes x 10,000 pods) unrecorded and staged, on k_simple's window
    (the default route) and forced onto k_schedule: chosen nodes, outcomes, the final node state
    and nextStartNodeIndex."""
    n_nodes, n_pods = 5000, 10000
    prof = _prof(pct)
    s = native.Synth(2, SEED_BASE + 2, n_nodes, n_pods)
    ch_o, res, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods, flags=abi.KSS_SCHED_GENERAL_KERNEL if kernel == "k_schedule" else 0)
    assert ctx.last_kernel() == kernel
    np.testing.assert_array_equal(chosen, ch_o)
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    assert ctx.next_start_node_index() == st["next_start"]
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    np.testing.assert_array_equal(g["pod_count"][:n_nodes], st["pod_count"][:n_nodes])
    ctx.close()


@pytest.mark.parametrize("geometry", ["xcd_local", "unrestricted", "one_shard", "three_shards", "chunks"])
@pytest.mark.parametrize("pct", [0, 12])
def test_k_simple_window_geometries(pct, geometry):
    """k_simple's window (simple_sync_win) in each of its shapes against the C oracle: the XCD-local
    grid (32 shards, per-wave mode), the unrestricted one (40 shards), one shard (no exchange, the
    cut ranked locally, per-thread mode), three shards of 1,000 nodes (per-thread mode), and several
    chunk launches (KSS static budget: 7 launches hand nextStartNodeIndex on through the device
    word).  The batch starts at a set cursor; two runs.  (A k_simple shard holds at most ~1,200
    nodes: 132 B of LDS per node slot, simple_lds_bytes.)"""
    n_nodes = {"one_shard": 1000, "three_shards": 3000}.get(geometry, 5000)
    n_pods, cursor = 1500, (777 if geometry == "one_shard" else 2321)
    prof = _prof(pct)
    s = native.Synth(2, SEED_BASE + 2, n_nodes, n_pods)
    ch_o, res, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes, record="meta", cursor=cursor)
    if geometry == "unrestricted":
        native.set_option("xcd", 0)
    elif geometry == "one_shard":
        native.set_option("shards", 1)
    elif geometry == "three_shards":
        native.set_option("shards", 3)
    elif geometry == "chunks":
        native.set_option("static_bytes", 4 * n_nodes * 220)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    for rep in range(2):
        ctx.reset()
        ctx.set_next_start_node_index(cursor)
        chosen = ctx.run_staged(n_pods)
        assert ctx.last_kernel() == "k_simple"
        want_shards = {"xcd_local": 32, "unrestricted": 40, "one_shard": 1, "three_shards": 3}.get(geometry)
        if want_shards:
            assert ctx.last_geometry()["shards"] == want_shards, ctx.last_geometry()
        if geometry == "chunks":
            assert ctx.last_timing()[1] >= 2 * 7
        np.testing.assert_array_equal(chosen, ch_o, err_msg=f"run {rep}")
        _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
        assert ctx.next_start_node_index() == st["next_start"]
        g = ctx.node_state()
        np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    ctx.close()


@pytest.mark.parametrize("n_nodes", [101, 180, 150])
def test_k_simple_window_small_and_saturating(n_nodes):
    """Window edges on k_simple: K = 100 of 101 / 180 nodes, and a cluster the batch saturates (pods
    become unschedulable, F <= K: every node visited, the cursor stays) -- chosen nodes, outcomes and
    the cursor against the oracle."""
    n_pods = 6000 if n_nodes == 150 else 400  # 150 nodes / 6,000 pods: 1,542 unschedulable
    prof = _prof(0)
    s = native.Synth(1, SEED_BASE + 1, n_nodes, n_pods)
    ch_o, res, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    assert ctx.last_kernel() == "k_simple"
    np.testing.assert_array_equal(chosen, ch_o)
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    assert ctx.next_start_node_index() == st["next_start"]
    if n_nodes == 150:
        assert (ch_o < 0).any()  # the batch saturates the cluster
    ctx.close()


def test_cursor_continues_across_batches_and_resets():
    """Two batches (pods [0, 300) then [300, 600) of one podset): the second starts where the
    first left nextStartNodeIndex; kss_reset_node_state starts it at 0 again; the setter
    moves it."""
    n_nodes, n_pods = 3000, 600
    prof = _prof(0)
    s = native.Synth(2, SEED_BASE + 2, n_nodes, n_pods)
    ch_o, _, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes, record=False)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    a = ctx.schedule_batch(s.pods, 300)
    mid = ctx.next_start_node_index()
    _, _, st1 = _oracle(prof, s.cluster, s.pods, 300, n_nodes, record=False)
    assert mid == st1["next_start"] and mid != 0
    np.testing.assert_array_equal(a, ch_o[:300])
    # the second half: the same podset with its first 300 pods removed (a new staging)
    from kss import abi as A
    import ctypes as C
    tail = A.PodSet.from_buffer_copy(s.pods)
    tail.n_pods = n_pods - 300
    tail.pods = C.cast(C.addressof(s.pods.pods.contents) + 300 * C.sizeof(A.Pod), C.POINTER(A.Pod))
    b = ctx.schedule_batch(tail, n_pods - 300)
    np.testing.assert_array_equal(b, ch_o[300:])
    assert ctx.next_start_node_index() == st["next_start"]
    ctx.reset()
    assert ctx.next_start_node_index() == 0
    ctx.set_next_start_node_index(1234)
    assert ctx.next_start_node_index() == 1234
    ch2, _, _ = _oracle(prof, s.cluster, s.pods, 50, n_nodes, record=False, cursor=1234)
    np.testing.assert_array_equal(ctx.schedule_batch(s.pods, 50), ch2)
    ctx.close()


@pytest.mark.parametrize("n_nodes", [100, 101, 180])
def test_min_feasible_nodes_edge(n_nodes):
    """The C1 edge: 100 nodes keep every node (numFeasibleNodesToFind's floor); from 101 nodes
    K = 100 < N and the search stops at the 101st feasible node when there is one; default
    profile, adaptive pct, every record."""
    n_pods = 200
    prof = _prof(0)
    s = native.Synth(1, SEED_BASE + 1, n_nodes, n_pods)
    ch_o, res, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes)
    ctx = native.Context(prof, max_pods_record=n_pods)
    ctx.load(s.cluster)
    np.testing.assert_array_equal(ctx.schedule_batch(s.pods, n_pods, record=True), ch_o)
    dropped = 0
    for j in range(n_pods):
        r = ctx.fetch_record(j)
        _record_equal(r, res, j, n_nodes)
        dropped += int((r.fail_detail[:n_nodes] == abi.KSS_PASS_NOT_KEPT).sum())
    if n_nodes == 100:
        assert dropped == 0  # K = N: the search never stops early
    if n_nodes == 180:
        assert dropped > 0
    assert ctx.next_start_node_index() == st["next_start"]
    ctx.close()


def test_spread_programs_and_name_sets():
    """Config-3 programs (PodTopologySpread PreScore sizes over the kept nodes, InterPodAffinity
    normalisation) and PreFilterResult sets of 120 and 30 nodes, pct 20, sharded, every record."""
    from test_oracle_crosscheck import with_name_sets
    from kss import synth
    nodes, bound, pods = synth.make_cluster(3, 900, 160)
    names = [n["metadata"]["name"] for n in nodes]
    pods = with_name_sets(pods, names, every=3, size=120)
    pods = with_name_sets(pods, names, every=7, size=30, seed=11)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    prof = _prof(20)
    N = cc.n_nodes
    ch_o, res, st = _oracle(prof, cc.as_struct(), cp.as_struct(), cp.n, N, n_classes=len(cc.classes),
                            n_terms=len(cc.terms))
    ctx = native.Context(prof, max_pods_record=cp.n)
    ctx.load(cc.as_struct())
    np.testing.assert_array_equal(ctx.schedule_batch(cp.as_struct(), cp.n, record=True,
                                                     flags=abi.KSS_SCHED_FORCE_MULTI_WG), ch_o)
    for j in range(cp.n):
        _record_equal(ctx.fetch_record(j), res, j, N)
    assert ctx.next_start_node_index() == st["next_start"]
    ctx.close()


def test_per_pod_api_advances_the_cursor():
    """kss_eval_pod + kss_commit pod after pod (the drop-in's PreFilter / Reserve) equals the
    batch: every evaluated cycle advances nextStartNodeIndex."""
    n_nodes, n_pods = 2000, 120
    prof = _prof(0)
    s = native.Synth(2, SEED_BASE + 2, n_nodes, n_pods)
    ch_o, res, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    for j in range(n_pods):
        r = ctx.eval_pod(s.pods, j)
        _record_equal(r, res, j, n_nodes)
        if r.chosen >= 0:
            ctx.commit(s.pods, j, r.chosen)
    assert ctx.next_start_node_index() == st["next_start"]
    ctx.close()


def test_service_grid_window():
    """The resident service grid: eval + commit pod after pod equals the oracle, the compact
    record's full re-evaluation (is_wide) repeats the cycle from the same cursor, and the
    cursor the grid leaves is the oracle's."""
    n_nodes, n_pods = 2000, 120
    prof = _prof(0)
    s = native.Synth(2, SEED_BASE + 2, n_nodes, n_pods)
    ch_o, res, st = _oracle(prof, s.cluster, s.pods, n_pods, n_nodes)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    for j in range(n_pods):
        v = ctx.service_eval(j) if j % 2 else ctx.service_eval_compact(j)
        if j % 2 == 0 and v.is_wide:
            v = v.wide
        if j % 2:
            _record_equal(v, res, j, n_nodes)
        else:
            m = res.meta(j)
            assert (v.chosen, v.n_feasible) == (m["chosen"], m["n_feasible"]), j
            np.testing.assert_array_equal(v.fail_detail[:n_nodes], res.fail_detail[j, :n_nodes], err_msg=str(j))
        if v.chosen >= 0:
            ctx.service_commit(j, v.chosen)
    ctx.service_stop()
    assert ctx.next_start_node_index() == st["next_start"]
    ctx.close()


def test_sweep_window():
    """Scenario sweep under pct 0: k_schedule per scenario, each scenario's cursor from 0 on
    every run, two runs equal to the oracle."""
    prof = _prof(0)
    syn = [native.Synth(5, SEED_BASE + 5 + 7919 * k, n, 150) for k, n in enumerate([300, 101, 700, 100, 250, 512])]
    sw = native.Sweep(prof, [x.cluster for x in syn], [x.pods for x in syn])
    assert sw.info()["kernel"] == "k_schedule"
    want = np.concatenate([_oracle(prof, x.cluster, x.pods, x.n_pods, x.n_nodes, record=False)[0] for x in syn])
    for rep in range(2):
        chosen, _ = sw.run()
        np.testing.assert_array_equal(chosen, want, err_msg=f"run {rep}")
    sw.close()
