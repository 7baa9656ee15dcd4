"""HIP path (libkss.so on gfx950) vs the CPU oracle: bit-exact filter verdicts, every
per-plugin raw and normalized score, totals, chosen nodes and the final node state.

Sizes are ones the oracle finishes in seconds; the full BASELINE sizes are in
test_gpu_scale.py.
"""
import json
import os

import numpy as np
import pytest

import k8s_oracle
import oracle_c
from kss import abi, native, synth
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "readme_known_answer.json")))


def _compare_records(ctx, res, chosen_o, n_pods, n_nodes):
    for j in range(n_pods):
        r = ctx.fetch_record(j)
        m = res.meta(j)
        assert r.chosen == m["chosen"], (j, r.chosen, m["chosen"])
        assert r.n_feasible == m["n_feasible"], j
        assert r.scored == m["scored"], j
        assert r.status == m["status"], j
        np.testing.assert_array_equal(r.fail_plugin[:n_nodes], res.fail_plugin[j, :n_nodes], err_msg=f"pod {j}")
        np.testing.assert_array_equal(r.fail_detail[:n_nodes], res.fail_detail[j, :n_nodes], err_msg=f"pod {j}")
        if m["scored"]:
            feas = res.fail_plugin[j, :n_nodes] == 0
            np.testing.assert_array_equal(r.raw[:, :n_nodes][:, feas], res.raw[j][:, :n_nodes][:, feas], err_msg=f"pod {j}")
            np.testing.assert_array_equal(r.norm[:, :n_nodes][:, feas], res.norm[j][:, :n_nodes][:, feas], err_msg=f"pod {j}")
            np.testing.assert_array_equal(r.total[:n_nodes][feas], res.total[j, :n_nodes][feas], err_msg=f"pod {j}")
            assert r.s.best_total == m["best_total"]


def _state_equal(ctx, st, n_nodes, n_classes, n_terms):
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    np.testing.assert_array_equal(g["nonzero"][:, :n_nodes], st["nonzero"][:, :n_nodes])
    np.testing.assert_array_equal(g["pod_count"][:n_nodes], st["pod_count"][:n_nodes])
    if n_classes:
        np.testing.assert_array_equal(g["class_count"][:n_classes], st["class_count"][:n_classes])
    if n_terms:
        np.testing.assert_array_equal(g["term_count"][:n_terms], st["term_count"][:n_terms])


MODES = {"auto": 0, "single": abi.KSS_SCHED_FORCE_SINGLE_WG, "multi": abi.KSS_SCHED_FORCE_MULTI_WG}


@pytest.mark.parametrize("mode", ["auto", "single", "multi"])
@pytest.mark.parametrize("config,n_nodes,n_pods", [
    (1, 100, 1000),   # C1 exactly (BASELINE configs[0])
    (2, 700, 400),
    (3, 300, 400),    # PTS + IPA
    (4, 500, 300),    # zone spread
    (5, 1000, 200),
    (1, 3, 50),       # tiny: single-feasible and unschedulable pods
    (3, 1500, 120),   # several nodes per lane
])
def test_schedule_batch_matches_oracle(config, n_nodes, n_pods, mode):
    """Single workgroup, forced multi-shard (granule exchanges) and the automatic geometry
    all give the oracle's results bit for bit."""
    prof = abi.default_profile()
    s = native.Synth(config, 0, n_nodes, n_pods)
    chosen_o, res, st = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record=True, threads=8,
                                          n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    ctx = native.Context(prof, max_pods_record=n_pods)
    ctx.load(s.cluster)
    chosen_g = ctx.schedule_batch(s.pods, n_pods, record=True, flags=MODES[mode])
    geo = ctx.last_geometry()
    if mode == "single":
        assert geo["shards"] == 1
    if mode == "multi" and n_nodes >= 4:
        assert geo["shards"] > 1
    np.testing.assert_array_equal(chosen_g, chosen_o)
    _compare_records(ctx, res, chosen_o, n_pods, n_nodes)
    _state_equal(ctx, st, n_nodes, s.cluster.n_classes, s.cluster.n_terms)


@pytest.mark.parametrize("mode", ["auto", "single", "multi"])
@pytest.mark.parametrize("config,n_nodes,n_pods", [
    (1, 100, 1000),   # C1 exactly
    (2, 700, 400),
    (5, 1000, 300),
    (1, 3, 50),       # tiny: single-feasible and unschedulable pods
    (2, 1500, 150),   # several nodes per lane
    (2, 5000, 120),   # C2 cluster
])
def test_compact_kernel_matches_oracle(config, n_nodes, n_pods, mode):
    """k_simple (register-resident rows, one speculative exchange per pod): chosen node,
    per-pod outcome (feasible count, scored, status, best total) and the final node state
    equal the oracle's."""
    if mode == "single" and n_nodes > 1024:
        pytest.skip("more nodes than one workgroup's LDS shard image holds")
    prof = abi.default_profile()
    s = native.Synth(config, 0, n_nodes, n_pods)
    chosen_o, res, st = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record=True, threads=8,
                                          n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    chosen_g = ctx.schedule_batch(s.pods, n_pods, flags=MODES[mode])
    assert ctx.last_kernel() == "k_simple"
    geo = ctx.last_geometry()
    if mode == "single":
        assert geo["shards"] == 1
    if mode == "multi" and n_nodes >= 4:
        assert geo["shards"] > 1
    np.testing.assert_array_equal(chosen_g, chosen_o)
    meta = ctx.fetch_meta(n_pods)
    for j in range(n_pods):
        m = res.meta(j)
        got = dict(chosen=meta[j, 0], n_feasible=meta[j, 1], scored=meta[j, 2], status=meta[j, 3])
        assert got == {k: m[k] for k in got}, (j, got, m)
        if m["scored"]:
            assert meta[j, 4] == m["best_total"], j
    _state_equal(ctx, st, n_nodes, s.cluster.n_classes, s.cluster.n_terms)


def test_compact_and_general_kernels_agree_at_c2_scale():
    prof = abi.default_profile()
    s = native.Synth(2, 0, 5000, 2000)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    a = ctx.run_staged(2000).copy()
    assert ctx.last_kernel() == "k_simple"
    st_a = ctx.node_state()
    ctx.reset()
    b = ctx.schedule_batch(s.pods, 2000, flags=abi.KSS_SCHED_GENERAL_KERNEL)
    assert ctx.last_kernel() == "k_schedule"
    np.testing.assert_array_equal(a, b)
    st_b = ctx.node_state()
    for k in st_a:
        np.testing.assert_array_equal(st_a[k], st_b[k])


def test_schedule_without_record_same_choices():
    prof = abi.default_profile()
    s = native.Synth(3, 0, 400, 300)
    chosen_o, _, st = oracle_c.schedule(prof, s.cluster, s.pods, 300, 400, record=False, threads=8,
                                        n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    np.testing.assert_array_equal(ctx.schedule_batch(s.pods, 300), chosen_o)
    _state_equal(ctx, st, 400, s.cluster.n_classes, s.cluster.n_terms)


def test_compiled_objects_path_and_annotations():
    """Objects -> host compiler -> GPU; annotations formatted lazily from HBM records equal the
    object-level oracle's store.go restatement byte for byte."""
    nodes, bound, pods = synth.make_cluster(3, 40, 80)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ctx = native.Context(abi.default_profile(), max_pods_record=cp.n)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    ctx.schedule_batch(cp.as_struct(), cp.n, record=True)
    o = k8s_oracle.Oracle(nodes, bound)
    for j in range(cp.n):
        want = o.annotations(o.schedule_one(pods[j]))
        got = ctx.format_annotations(ctx.fetch_record(j))
        assert got == want, j


def test_readme_known_answer_on_gpu():
    cc, cp, _ = compile_cluster(GOLD["nodes"], (), [GOLD["pod"]])
    ctx = native.Context(abi.default_profile(), max_pods_record=1)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    r = ctx.eval_pod(cp.as_struct(), 0)
    ann = ctx.format_annotations(r)
    for k, v in GOLD["expected"].items():
        if isinstance(v, dict):
            assert json.loads(ann[k]) == v, k
        else:
            assert ann[k] == v, k


GOLD2 = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "extender_known_answer.json")))


def _check_ann(ann, exp):
    from test_oracle_known_answer import check_annotations
    check_annotations(ann, exp)


def test_extender_doc_known_answer_on_gpu():
    """simulator/docs/plugin-extender.md:80-109 on the device: (a) the drop-in per-pod call
    on the snapshot with node-282x7 already holding a pod; (b) the two pods as a sequential
    batch on the empty nodes (the first one's AssumePod happens on the device)."""
    cc, cp, _ = compile_cluster(GOLD2["nodes"], GOLD2["bound"], [GOLD2["pod"]])
    ctx = native.Context(abi.default_profile(), max_pods_record=2)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    _check_ann(ctx.format_annotations(ctx.eval_pod(cp.as_struct(), 0)), GOLD2["expected"])
    ctx.close()
    first = dict(GOLD2["bound"][0], spec={k: v for k, v in GOLD2["bound"][0]["spec"].items() if k != "nodeName"})
    cc, cp, _ = compile_cluster(GOLD2["nodes"], (), [first, GOLD2["pod"]])
    ctx = native.Context(abi.default_profile(), max_pods_record=2)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    chosen = ctx.schedule_batch(cp.as_struct(), 2, record=True)
    assert [cc.node_names[c] for c in chosen] == ["node-282x7", "node-gp9t4"]
    _check_ann(ctx.format_annotations(ctx.fetch_record(1)), GOLD2["expected"])
    ctx.close()


def test_eval_pod_commit_rollback():
    prof = abi.default_profile()
    s = native.Synth(3, 0, 200, 20)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    before = ctx.node_state()
    for j in range(5):
        want = oracle_c.Results(1, 200)
        # oracle on the current committed state: schedule pods [0, j] and compare pod j
        ch, res, _ = oracle_c.schedule(prof, s.cluster, s.pods, j + 1, 200, threads=8,
                                       n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
        r = ctx.eval_pod(s.pods, j)
        assert r.chosen == ch[j]
        np.testing.assert_array_equal(r.fail_plugin[:200], res.fail_plugin[j, :200])
        if r.chosen >= 0:
            ctx.commit(s.pods, j, r.chosen)
    # roll everything back -> original state
    ch, _, _ = oracle_c.schedule(prof, s.cluster, s.pods, 5, 200, n_classes=s.cluster.n_classes,
                                 n_terms=s.cluster.n_terms)
    for j in range(5):
        if ch[j] >= 0:
            ctx.rollback(s.pods, j, int(ch[j]))
    after = ctx.node_state()
    for k in before:
        np.testing.assert_array_equal(before[k], after[k])


def test_eval_pod_view_equals_eval_pod():
    """kss_eval_pod_view (arrays in place in the pinned staging) returns what kss_eval_pod
    copies out, and only the fields asked for."""
    s = native.Synth(3, 0, 300, 12)
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    N = 300
    for j in range(12):
        r = ctx.eval_pod(s.pods, j)
        want = {k: getattr(r, k).copy() for k in ("fail_plugin", "fail_detail", "raw", "norm", "total")}
        v = ctx.eval_pod_view(s.pods, j)
        assert (v.chosen, v.n_feasible, v.scored, v.status) == (r.chosen, r.n_feasible, r.scored, r.status)
        np.testing.assert_array_equal(v.fail_plugin, want["fail_plugin"][:N])
        np.testing.assert_array_equal(v.fail_detail, want["fail_detail"][:N])
        ok = want["fail_plugin"][:N] == abi.KSS_F_PASS
        np.testing.assert_array_equal(v.raw[:, ok], want["raw"][:, :N][:, ok])
        if r.scored:
            np.testing.assert_array_equal(v.norm[:, ok], want["norm"][:, :N][:, ok])
            np.testing.assert_array_equal(v.total[ok], want["total"][:N][ok])
        slim = ctx.eval_pod_view(s.pods, j, abi.KSS_FIELD_FAIL | abi.KSS_FIELD_TOTAL)
        assert slim.raw is None and slim.norm is None and slim.fail_detail is None
        np.testing.assert_array_equal(slim.fail_plugin, want["fail_plugin"][:N])
        if r.chosen >= 0:
            ctx.commit(s.pods, j, r.chosen)
    ctx.close()


@pytest.mark.parametrize("config,sizes,n_pods", [
    (5, [300] * 12, 150),            # k_simple sweep, one workgroup per scenario
    (5, [1000] * 8, 200),            # C5 scenario size
    (2, [100, 700, 1000, 3], 120),   # ragged scenario sizes in one launch
    (1, [3] * 5, 30),                # single-feasible / unschedulable pods
    (4, [200] * 6, 100),             # zone spread programs: k_schedule sweep
])
def test_scenarios_match_oracle_per_scenario(config, sizes, n_pods):
    prof = abi.default_profile()
    syn = [native.Synth(config, 0x5EED0000 + config + 7919 * sc, n, n_pods) for sc, n in enumerate(sizes)]
    chosen, ms = native.schedule_scenarios(prof, [x.cluster for x in syn], [x.pods for x in syn])
    off = 0
    for x in syn:
        ch, _, _ = oracle_c.schedule(prof, x.cluster, x.pods, x.n_pods, x.n_nodes, record=False, threads=8,
                                     n_classes=x.cluster.n_classes, n_terms=x.cluster.n_terms)
        np.testing.assert_array_equal(chosen[off:off + x.n_pods], ch)
        off += x.n_pods
    assert ms > 0


def test_invalid_program_is_rejected_not_run():
    s = native.Synth(1, 0, 50, 10)
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    bad = abi.PodSet.from_buffer_copy(bytes(s.pods))
    bad.n_ints = 0
    bad.n_reqs = 0  # requirement offsets now out of range
    with pytest.raises(native.KssError):
        ctx.schedule_batch(bad, 10)


@pytest.mark.parametrize("config,n_pods", [(2, 300), (4, 200)])
def test_c2_scale_sharded_matches_oracle(config, n_pods):
    """5,000 nodes (BASELINE C2 cluster) on the automatic multi-shard geometry: chosen nodes
    and final node state equal the oracle's for the first n_pods pods."""
    prof = abi.default_profile()
    n_nodes = 5000
    s = native.Synth(config, 0, n_nodes, n_pods)
    chosen_o, _, st = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record=False, threads=8,
                                        n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen_g = ctx.run_staged(n_pods)
    assert ctx.last_geometry()["shards"] > 1
    np.testing.assert_array_equal(chosen_g, chosen_o)
    _state_equal(ctx, st, n_nodes, s.cluster.n_classes, s.cluster.n_terms)
    # reset + replay gives the same placements (what-if replays)
    ctx.reset()
    np.testing.assert_array_equal(ctx.run_staged(n_pods), chosen_o)


def _podset_from(ps, first):
    """View of pods [first, n) of a podset (the pools are shared)."""
    import ctypes as C
    v = abi.PodSet.from_buffer_copy(ps)
    v.n_pods = ps.n_pods - first
    v.pods = C.cast(C.addressof(ps.pods.contents) + first * C.sizeof(abi.Pod), C.POINTER(abi.Pod))
    return v


def test_external_binds_through_node_and_count_deltas():
    """Pods bound outside this scheduler reach the snapshot through kss_apply_node_delta (node
    rows) and kss_apply_count_delta (class rows added, term rows overwritten): the state then
    equals the oracle's after those pods, and the following pods schedule as the oracle's
    uninterrupted run does."""
    prof = abi.default_profile()
    n_nodes, n_pods, n0 = 300, 160, 60
    s = native.Synth(3, 0, n_nodes, n_pods)
    ncl, nt = s.cluster.n_classes, s.cluster.n_terms
    chosen_all, _, _ = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, threads=8, n_classes=ncl,
                                         n_terms=nt)
    _, _, st0 = oracle_c.schedule(prof, s.cluster, s.pods, n0, n_nodes, threads=8, n_classes=ncl, n_terms=nt)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    orig = ctx.node_state()
    N = n_nodes
    moved = ((st0["requested"][:, :N] != orig["requested"][:, :N]).any(0) |
             (st0["nonzero"][:, :N] != orig["nonzero"][:, :N]).any(0) | (st0["pod_count"][:N] != orig["pod_count"][:N]))
    rows = np.nonzero(moved)[0]
    assert len(rows) > 20
    ctx.apply_node_delta(rows, st0["requested"][:, rows].T, st0["nonzero"][:, rows].T, st0["pod_count"][rows])
    dc = st0["class_count"][:ncl, :N].astype(np.int64) - orig["class_count"][:ncl, :N]
    r, n = np.nonzero(dc)
    ctx.apply_count_delta(n, r, dc[r, n])
    tdiff = st0["term_count"][:nt, :N] != orig["term_count"][:nt, :N]
    r, n = np.nonzero(tdiff)
    ctx.apply_count_delta(n, ncl + r, st0["term_count"][:nt, :N][r, n], overwrite=True)
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :N], st0["requested"][:, :N])
    np.testing.assert_array_equal(g["nonzero"][:, :N], st0["nonzero"][:, :N])
    np.testing.assert_array_equal(g["pod_count"][:N], st0["pod_count"][:N])
    np.testing.assert_array_equal(g["class_count"][:ncl], st0["class_count"][:ncl])
    np.testing.assert_array_equal(g["term_count"][:nt], st0["term_count"][:nt])
    chosen = ctx.schedule_batch(_podset_from(s.pods, n0), n_pods - n0)
    np.testing.assert_array_equal(chosen, chosen_all[n0:])
    ctx.close()
