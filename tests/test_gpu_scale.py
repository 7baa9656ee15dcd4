"""Full-size GPU parity: the BASELINE configurations and kernel geometries the smaller
cases in test_gpu_parity.py do not reach, compared bit-exactly with the C oracle.

  * C3 (5,000 nodes, 3 zones, PodTopologySpread + InterPodAffinity) with every per-node
    record (verdict, failure detail, raw / normalized scores, totals);
  * the whole C2 batch the bench times (5,000 nodes x 10,000 pods on k_simple);
  * k_simple at 100,000 nodes: 128 shards x 4 node slots per lane, i.e. both chunks of the
    shard-granule sweep (kss_simple.cuh simple_exchange, SX_CHUNKS);
  * C4's recipe (100,000 nodes, zone DoNotSchedule spread) on one GPU (k_spread and
    k_schedule, 256 shards) and the node-axis kernels at 100,000 rows, world 1;
  * a 64-scenario slice of the C5 sweep (1,000 nodes x 1,000 pods each).
"""
import os

import numpy as np
import pytest

import oracle_c
from kss import abi, native, nodeaxis
from kss.synth import SEED_BASE

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def _oracle(prof, s, n_pods, record=False):
    return oracle_c.schedule(prof, s.cluster, s.pods, n_pods, s.n_nodes, record=record, threads=THREADS,
                             n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)


def _meta_equal(meta, res_or_chosen, n):
    for j in range(n):
        m = res_or_chosen.meta(j)
        got = dict(chosen=meta[j, 0], n_feasible=meta[j, 1], scored=meta[j, 2], status=meta[j, 3])
        assert got == {k: m[k] for k in got}, (j, got, m)
        if m["scored"]:
            assert meta[j, 4] == m["best_total"], j


def _state_equal(ctx, st, n_nodes, n_classes, n_terms):
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    np.testing.assert_array_equal(g["nonzero"][:, :n_nodes], st["nonzero"][:, :n_nodes])
    np.testing.assert_array_equal(g["pod_count"][:n_nodes], st["pod_count"][:n_nodes])
    if n_classes:
        np.testing.assert_array_equal(g["class_count"][:n_classes], st["class_count"][:n_classes])
    if n_terms:
        np.testing.assert_array_equal(g["term_count"][:n_terms], st["term_count"][:n_terms])


def test_c3_full_cluster_with_records():
    """BASELINE configs[2]: 5,000 nodes, 500 pods, every per-node record of every pod."""
    prof = abi.default_profile()
    n_nodes, n_pods = 5000, 500
    s = native.Synth(3, 0, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record=True)
    ctx = native.Context(prof, max_pods_record=n_pods)
    ctx.load(s.cluster)
    chosen = ctx.schedule_batch(s.pods, n_pods, record=True)
    assert ctx.last_geometry()["shards"] > 1
    np.testing.assert_array_equal(chosen, chosen_o)
    for j in range(n_pods):
        r = ctx.fetch_record(j)
        m = res.meta(j)
        assert (r.chosen, r.n_feasible, r.scored, r.status) == (m["chosen"], m["n_feasible"], m["scored"],
                                                                m["status"]), j
        np.testing.assert_array_equal(r.fail_plugin[:n_nodes], res.fail_plugin[j], err_msg=f"pod {j}")
        np.testing.assert_array_equal(r.fail_detail[:n_nodes], res.fail_detail[j], err_msg=f"pod {j}")
        if m["scored"]:
            feas = res.fail_plugin[j] == 0
            np.testing.assert_array_equal(r.raw[:, feas], res.raw[j][:, feas], err_msg=f"pod {j}")
            np.testing.assert_array_equal(r.norm[:, feas], res.norm[j][:, feas], err_msg=f"pod {j}")
            np.testing.assert_array_equal(r.total[feas], res.total[j][feas], err_msg=f"pod {j}")
            assert r.s.best_total == m["best_total"], j
    _state_equal(ctx, st, n_nodes, s.cluster.n_classes, s.cluster.n_terms)
    ctx.close()


def test_c3_full_batch_no_record():
    """C3 5,000 nodes x 2,000 pods through the resident path (chosen, outcomes, final
    state including the class / term counts that commits update)."""
    prof = abi.default_profile()
    n_nodes, n_pods = 5000, 2000
    s = native.Synth(3, 0, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    np.testing.assert_array_equal(ctx.run_staged(n_pods), chosen_o)
    assert ctx.last_kernel() == "k_spread"
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, s.cluster.n_classes, s.cluster.n_terms)
    ctx.close()


def test_c2_full_batch_matches_oracle():
    """BASELINE configs[1] exactly as bench.py times it: 5,000 nodes x 10,000 pods from the
    initial snapshot, resident inputs, k_simple."""
    prof = abi.default_profile()
    n_nodes, n_pods = 5000, 10000
    s = native.Synth(2, SEED_BASE + 2, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    for rep in range(2):  # the bench's reset + replay
        ctx.reset()
        chosen = ctx.run_staged(n_pods)
        assert ctx.last_kernel() == "k_simple"
        np.testing.assert_array_equal(chosen, chosen_o, err_msg=f"replay {rep}")
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, 0, 0)
    ctx.close()


def test_k_simple_100k_nodes_two_sweep_chunks():
    """100,000 nodes: 128 k_simple shards (both 64-shard chunks of the granule sweep) with
    4 node slots per lane."""
    prof = abi.default_profile()
    n_nodes, n_pods = 100000, 200
    s = native.Synth(2, SEED_BASE + 4, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    geo = ctx.last_geometry()
    assert ctx.last_kernel() == "k_simple"
    assert geo["shards"] > 64 and geo["nodes_per_lane"] > 1, geo
    np.testing.assert_array_equal(chosen, chosen_o)
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, 0, 0)
    ctx.close()


@pytest.mark.parametrize("shards", [65, 100])
def test_k_simple_forced_shards_above_one_chunk(shards, monkeypatch):
    """KSS_SHARDS forces W > 64 on a 20,000-node cluster (second sweep chunk, ragged)."""
    native.set_option("shards", str(shards))
    prof = abi.default_profile()
    n_nodes, n_pods = 20000, 300
    s = native.Synth(2, 0, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    assert ctx.last_kernel() == "k_simple"
    assert ctx.last_geometry()["shards"] == shards
    np.testing.assert_array_equal(chosen, chosen_o)
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, 0, 0)
    ctx.close()


@pytest.mark.parametrize("kernel,n_pods", [("k_spread", 200), ("k_schedule", 200), ("k_spread", 2000)])
def test_c4_recipe_on_one_gpu(kernel, n_pods, monkeypatch):
    """BASELINE configs[3]'s recipe (100,000 nodes, zone DoNotSchedule spread) on one GPU at
    256 shards: k_spread, and the general kernel (KSS_NO_SPREAD).  At 2,000 pods the batch
    reads ~100 count rows, which fit only because the LDS slots are strided by the 391-node
    shard, not by threads x slots per lane."""
    if kernel == "k_schedule":
        native.set_option("no_spread", "1")
    prof = abi.default_profile()
    n_nodes = 100000
    s = native.Synth(4, 0, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    assert ctx.last_kernel() == kernel
    np.testing.assert_array_equal(chosen, chosen_o)
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, s.cluster.n_classes, 0)
    ctx.close()


def test_c4_bench_shape_many_chunks(monkeypatch):
    """The shape bench.py's C4 leg times: unsplit k_spread on BASELINE configs[3]'s recipe
    and seed at 100,000 nodes over several k_static chunks (the bench runs 8 per step);
    KSS_STATIC_BYTES forces 4 chunks of 1,250 pods, so node state and count rows cross three
    launch boundaries.  Chosen nodes, per-pod outcomes and the final state with the class
    counts against the C oracle."""
    n_nodes, n_pods, per_chunk = 100000, 5000, 1250
    native.set_option("static_bytes", str(4 * n_nodes * per_chunk))
    prof = abi.default_profile()
    s = native.Synth(4, SEED_BASE + 4, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    assert ctx.last_kernel() == "k_spread"
    assert ctx.last_timing()[1] == 2 * (n_pods // per_chunk)  # k_static + k_spread per chunk
    np.testing.assert_array_equal(chosen, chosen_o)
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, s.cluster.n_classes, 0)
    ctx.close()


def test_nodeaxis_100k_rows_world1():
    n_nodes, n_pods = 100000, 300
    prof = abi.default_profile()
    s = native.Synth(2, SEED_BASE + 4, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    sch = nodeaxis.NodeAxisScheduler(s.cluster, s.pods, prof, device=0)
    chosen = sch.schedule().cpu().numpy()
    np.testing.assert_array_equal(chosen, chosen_o)
    _meta_equal(sch.meta(n_pods), res, n_pods)
    g = sch.node_state()
    np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    np.testing.assert_array_equal(g["pod_count"][:n_nodes], st["pod_count"][:n_nodes])
    sch.close()


def test_c5_sweep_64_scenarios():
    """64 scenarios of the C5 sweep (1,000 nodes x 1,000 pods each, seed per scenario) in
    one launch, each against its own oracle run."""
    prof = abi.default_profile()
    syn = [native.Synth(5, SEED_BASE + 5 + 7919 * k, 1000, 1000) for k in range(64)]
    chosen, ms = native.schedule_scenarios(prof, [x.cluster for x in syn], [x.pods for x in syn])
    assert ms > 0
    off = 0
    for k, x in enumerate(syn):
        ch, _, _ = _oracle(prof, x, x.n_pods)
        np.testing.assert_array_equal(chosen[off:off + x.n_pods], ch, err_msg=f"scenario {k}")
        off += x.n_pods


def test_sweep_resident_reruns_match_oracle():
    """kss_sweep: staged once (one upload), run twice; every run restores the snapshots on
    the device, so both equal the oracle.  Ragged sizes in one sweep."""
    prof = abi.default_profile()
    syn = [native.Synth(2, SEED_BASE + 2 + 7919 * k, n, 150) for k, n in enumerate([1000, 37, 700, 1000, 3, 512])]
    sw = native.Sweep(prof, [x.cluster for x in syn], [x.pods for x in syn])
    assert sw.info()["kernel"] == "k_simple"
    want = np.concatenate([_oracle(prof, x, x.n_pods)[0] for x in syn])
    for rep in range(2):
        chosen, ms = sw.run()
        assert ms > 0
        np.testing.assert_array_equal(chosen, want, err_msg=f"run {rep}")
    sw.close()


def test_c5_sweep_forced_chunks_three_reruns(monkeypatch):
    """C5's shape (64 scenarios x 1,000 nodes x 1,000 pods) with KSS_STATIC_BYTES forcing four
    k_static chunks of 300 pods: every rerun restores all scenarios' node state with the reset
    kernel (no runtime copy) and the chunks hand node state over in HBM; three runs, each equal
    to the oracle scenario by scenario."""
    native.set_option("static_bytes", str(4 * 64 * 1000 * 300))
    prof = abi.default_profile()
    syn = [native.Synth(5, SEED_BASE + 5 + 7919 * k, 1000, 1000) for k in range(64)]
    sw = native.Sweep(prof, [x.cluster for x in syn], [x.pods for x in syn])
    assert sw.info()["kernel"] == "k_simple"
    want = [_oracle(prof, x, x.n_pods)[0] for x in syn]
    for rep in range(3):
        chosen, _ = sw.run()
        off = 0
        for k, x in enumerate(syn):
            np.testing.assert_array_equal(chosen[off:off + x.n_pods], want[k], err_msg=f"run {rep} scenario {k}")
            off += x.n_pods
    sw.close()


def test_sweep_odd_chunk_mixed_node_parity(monkeypatch):
    """An odd chunk (37 pods) over scenarios with odd and even node counts: each scenario's
    static words start at a 16-byte boundary, so k_static's paired 8-byte stores stay aligned
    (ADVICE r4); 151 pods, two runs."""
    sizes = [1001, 37, 700, 999, 3, 512, 64]
    native.set_option("static_bytes", str(4 * sum(sizes) * 37))
    prof = abi.default_profile()
    syn = [native.Synth(2, SEED_BASE + 2 + 7919 * k, n, 151) for k, n in enumerate(sizes)]
    sw = native.Sweep(prof, [x.cluster for x in syn], [x.pods for x in syn])
    assert sw.info()["kernel"] == "k_simple"
    want = np.concatenate([_oracle(prof, x, x.n_pods)[0] for x in syn])
    for rep in range(2):
        chosen, _ = sw.run()
        np.testing.assert_array_equal(chosen, want, err_msg=f"run {rep}")
    sw.close()


def _custom_profile():
    """MostAllocated over cpu:3 / memory:2 (weight sum 5), BalancedAllocation over three
    resources (the standard-deviation branch), non-default plugin weights."""
    prof = abi.default_profile()
    prof.fit_strategy = abi.KSS_FIT_MOST_ALLOCATED
    prof.fit_weight[0], prof.fit_weight[1] = 3, 2
    prof.ba_n = 3
    prof.ba_res[2] = abi.KSS_RES_EPHEMERAL
    prof.weight[abi.KSS_S_NODE_AFFINITY] = 5
    prof.weight[abi.KSS_S_TAINT_TOLERATION] = 1
    prof.weight[abi.KSS_S_BALANCED_ALLOCATION] = 4
    return prof


@pytest.mark.parametrize("n_nodes,n_pods", [(5000, 1500), (700, 400)])
def test_k_simple_custom_profile_matches_oracle(n_nodes, n_pods):
    prof = _custom_profile()
    s = native.Synth(2, 0, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    np.testing.assert_array_equal(ctx.run_staged(n_pods), chosen_o)
    assert ctx.last_kernel() == "k_simple"
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, 0, 0)
    ctx.close()


def test_k_simple_small_static_chunks(monkeypatch):
    """KSS_STATIC_BYTES forces the static words into many chunks (one k_static + one
    k_simple launch each, node state carried in HBM): same result as one chunk."""
    native.set_option("static_bytes", str(4 * 3000 * 37))  # 37 pods per chunk
    prof = abi.default_profile()
    n_nodes, n_pods = 3000, 400
    s = native.Synth(2, 0, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    np.testing.assert_array_equal(ctx.run_staged(n_pods), chosen_o)
    assert ctx.last_timing()[1] == 2 * ((n_pods + 36) // 37)
    _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
    _state_equal(ctx, st, n_nodes, 0, 0)
    ctx.close()


@pytest.mark.parametrize("config,kernel", [(2, "k_simple"), (3, "k_spread")])
@pytest.mark.parametrize("mode", ["forced_fallback", "xcd_off"])
def test_xcd_local_fallback_and_off(config, kernel, mode):
    """The XCD-local grid's fallback: when XCD 0 does not get W workgroups the launch
    fails with err 3 before touching any state and the host runs it again unrestricted.
    forced_fallback: kss_set_option("xcd_force_fallback") makes every XCD-local launch report
    failed placement, so the unrestricted rerun schedules the batch (counted in fallbacks);
    xcd_off: kss_set_option("xcd", 0), no XCD-local launch at all.  Both equal the oracle."""
    prof = abi.default_profile()
    n_nodes, n_pods = 5000, 400
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    chosen_o, res, st = _oracle(prof, s, n_pods, record="meta")
    native.set_option("xcd_force_fallback" if mode == "forced_fallback" else "xcd", 1 if mode == "forced_fallback" else 0)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    for rep in range(2):
        ctx.reset()
        chosen = ctx.run_staged(n_pods)
        assert ctx.last_kernel() == kernel
        xl = ctx.last_xcd_local()
        if mode == "forced_fallback":
            assert xl == {"used": 1, "fallbacks": 1}, xl
        else:
            assert xl["used"] == 0 and xl["fallbacks"] == 0, xl
        np.testing.assert_array_equal(chosen, chosen_o, err_msg=f"run {rep}")
        _meta_equal(ctx.fetch_meta(n_pods), res, n_pods)
        _state_equal(ctx, st, n_nodes, s.cluster.n_classes, s.cluster.n_terms)
    ctx.close()
    s.close()
