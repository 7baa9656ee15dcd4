"""Nominated pods on the device (kss_nominate / kss_clear_nomination / kss_remove_bound):
RunFilterPluginsWithNominatedPods, PreferNominatedNode and DeleteNominatedPodIfExists on k_schedule
(batches and the per-pod API) and in the PostFilter dry run (k_preempt), against the oracles:

  * the hand-derived fixture (tests/nominated_fixtures.py) per pod through kss_eval_pod + kss_commit;
  * recorded batches with nominees inside and after the batch against the C oracle's
    kss_oracle_schedule_n: every per-node verdict and detail, scores, outcomes, the nominations left,
    the final node state -- default profile, spread / inter-pod programs, the window (pct 30), one
    workgroup and the sharded grid;
  * saturated sequences with preemption: every unschedulable pod's PostFilter
    nominates a node, its victims are deleted (kss_remove_bound), lower-priority nominations on that
    node are cleared, the pod is nominated and retried after the queue; lower-priority pods that
    follow see the nominee -- statuses, nominated nodes, victims and chosen nodes equal
    oracle/k8s_preemption.schedule_with_nominations."""
import copy
import random

import numpy as np
import pytest

import k8s_oracle as ko
import k8s_preemption as kp
import nominated_fixtures as nf
import oracle_c
import preempt_fixtures as pf
from kss import abi, native, synth
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu

STATUS = {abi.KSS_PREEMPT_NOMINATED: "nominated", abi.KSS_PREEMPT_NO_CANDIDATE: "no_candidate",
          abi.KSS_PREEMPT_NOT_ELIGIBLE: "not_eligible", abi.KSS_PREEMPT_SCHEDULABLE: "schedulable"}
FILTER_CODE = {name: i for i, name in enumerate(abi.FILTER_PLUGINS) if name}


def _ctx(cc, prof=None, record=1):
    ctx = native.Context(prof or abi.default_profile(), max_pods_record=record)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    return ctx


def test_fixture_per_pod():
    nodes, bound, pods, noms, expect = nf.fixture()
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ps = cp.as_struct()
    idx = {n: i for i, n in enumerate(cc.node_names)}
    ctx = _ctx(cc)
    for j, n in noms:
        ctx.nominate(ps, j, idx[n])
    assert ctx.nominations() == [(j, idx[n]) for j, n in noms]
    for j, want in expect:
        r = ctx.eval_pod(ps, j)
        got = cc.node_names[r.chosen] if r.chosen >= 0 else None
        assert got == want["selected"], (j, got, want)
        for node, plugin in want.get("fail", {}).items():
            assert int(r.fail_plugin[idx[node]]) == (0 if plugin is None else FILTER_CODE[plugin]), (j, node)
        if "evaluated" in want:
            ev = sorted(cc.node_names[i] for i in range(cc.n_nodes) if r.fail_plugin[i] != abi.KSS_F_NOT_EVALUATED)
            assert ev == want["evaluated"], j
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
        if "nominated_left" in want:
            assert sorted(cp.names[q][1] for q, _ in ctx.nominations()) == want["nominated_left"], j
    ctx.close()


def _with_priorities(pods, seed, levels=(0, 0, 10, 100, 1000)):
    rnd = random.Random(seed)
    out = []
    for p in pods:
        p = copy.deepcopy(p)
        p["spec"]["priority"] = rnd.choice(levels)
        out.append(p)
    return out


def _noms(pods, n_nodes, n_run, seed, inside, outside):
    rnd = random.Random(seed)
    out = [(j, rnd.randrange(n_nodes)) for j in rnd.sample(range(n_run), inside)]
    for j in rnd.sample(range(n_run, len(pods)), outside):
        pods[j]["spec"]["priority"] = 1000
        out.append((j, rnd.randrange(n_nodes)))
    return out


CASES = {  # name: (cluster recipe, nodes, pods, pods run, nominations inside, after)
    "default": (lambda: synth.make_cluster(1, 300, 260), 300, 200, 6, 10),
    "small": (lambda: synth.make_cluster(1, 40, 160), 40, 120, 4, 8),
    "spread_ipa": (lambda: synth.make_cluster(3, 120, 200), 120, 150, 6, 12),
}


@pytest.mark.parametrize("pct", [100, 30])
@pytest.mark.parametrize("flags", [0, abi.KSS_SCHED_FORCE_SINGLE_WG])
@pytest.mark.parametrize("case", sorted(CASES))
def test_batch_matches_c_oracle(case, flags, pct):
    make, n_nodes, n_run, inside, outside = CASES[case]
    nodes, bound, pods = make()
    pods = _with_priorities(pods, 17)
    noms = _noms(pods, n_nodes, n_run, 17, inside, outside)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    ch_o, res, st = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), n_run, cc.n_nodes, threads=8,
                                      n_classes=len(cc.classes), n_terms=len(cc.terms), nominations=noms)
    ps = cp.as_struct()
    ctx = _ctx(cc, prof, record=n_run)
    for j, n in noms:
        ctx.nominate(ps, j, n)
    chosen = ctx.schedule_batch(ps, n_run, record=True, flags=flags)
    assert ctx.last_kernel() == "k_schedule"
    N = cc.n_nodes
    for j in range(n_run):
        r = ctx.fetch_record(j)
        np.testing.assert_array_equal(r.fail_plugin[:N], res.fail_plugin[j, :N], err_msg=f"pod {j} verdicts")
        np.testing.assert_array_equal(r.fail_detail[:N], res.fail_detail[j, :N], err_msg=f"pod {j} details")
        m = res.meta(j)
        assert (r.chosen, r.n_feasible, r.scored, r.status) == (m["chosen"], m["n_feasible"], m["scored"], m["status"]), j
        if m["scored"]:
            kept = (res.fail_plugin[j, :N] == 0) & (res.fail_detail[j, :N] != abi.KSS_PASS_NOT_KEPT)
            np.testing.assert_array_equal(r.raw[:, :N][:, kept], res.raw[j][:, :N][:, kept], err_msg=f"pod {j} raw")
            np.testing.assert_array_equal(r.total[:N][kept], res.total[j, :N][kept], err_msg=f"pod {j} total")
    np.testing.assert_array_equal(chosen, ch_o)
    assert ctx.nominations() == st["nominations"]
    assert ctx.next_start_node_index() == st["next_start"]
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :N], st["requested"][:, :N])
    ctx.close()


@pytest.mark.parametrize("uid", [False, True])
def test_per_pod_equals_batch(uid):
    """kss_eval_pod + kss_commit per pod gives the batch's choices and nominator (the pod's identity
    is its podset index on both paths, or the caller's uid)."""
    make, n_nodes, n_run, inside, outside = CASES["spread_ipa"]
    nodes, bound, pods = make()
    pods = _with_priorities(pods, 23)
    noms = _noms(pods, n_nodes, n_run, 23, inside, outside)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    if uid:
        cp.pods["uid"] = 1000 + np.arange(cp.n, dtype=np.int32)
    ps = cp.as_struct()
    a = _ctx(cc)
    for j, n in noms:
        a.nominate(ps, j, n)
    want = a.schedule_batch(ps, n_run)
    left = a.nominations()
    a.close()
    b = _ctx(cc)
    for j, n in noms:
        b.nominate(ps, j, n)
    got = []
    for j in range(n_run):
        r = b.eval_pod(ps, j)
        got.append(r.chosen)
        if r.chosen >= 0:
            b.commit(ps, j, r.chosen)
    assert got == list(want)
    assert b.nominations() == left
    if uid:
        assert {q for q, _ in left} <= {1000 + j for j, _ in noms}
        for q, _ in left:
            b.clear_nomination(ps, q - 1000)
        assert b.nominations() == []
    b.close()


def _oracle_seq(nodes, bound, pods):
    o, out = kp.schedule_with_nominations(nodes, bound, pods)
    res = []
    for j, r, pre in out:
        if r["selected"] is not None:
            res.append((j, "scheduled", ko._name(o.nodes[r["selected"]]), []))
        else:
            nom = ko._name(o.nodes[pre["nominated"]]) if pre["nominated"] is not None else None
            res.append((j, pre["status"], nom, [v[1] for v in pre["victims"]]))
    return res


def _device_seq(nodes, bound, pods):
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ps = cp.as_struct()
    ctx = _ctx(cc)
    ctx.load_bound(cc.as_boundset())
    prio = [ko.pod_priority(p) for p in pods]

    def victim_name(v):
        return cc.bound_names[v][1] if v >= 0 else cp.names[-1 - v][1]

    queue, tries, out = list(range(cp.n)), [0] * cp.n, []
    while queue:
        j = queue.pop(0)
        r = ctx.eval_pod(ps, j)
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
            out.append((j, "scheduled", cc.node_names[r.chosen], []))
            continue
        pre = ctx.postfilter_pod(ps, j)
        st = STATUS[pre["status"]]
        nom = cc.node_names[pre["nominated"]] if pre["nominated"] >= 0 else None
        out.append((j, st, nom, [victim_name(v) for v in pre["victims"]]))
        if st == "nominated":
            node = pre["nominated"]
            ctx.remove_bound(pre["victims"])  # prepareCandidate deletes them; the informer removes them
            for q, n in ctx.nominations():
                if n == node and prio[q] < prio[j]:
                    ctx.clear_nomination(ps, q)
            ctx.nominate(ps, j, node)
            if tries[j] < 1:
                tries[j] += 1
                queue.append(j)
        elif st == "no_candidate":
            ctx.clear_nomination(ps, j)
    ctx.close()
    return out


@pytest.mark.parametrize("seed,n_nodes,n_pods", [(1, 60, 40), (2, 60, 50), (3, 200, 60), (6, 120, 80)])
def test_saturated_sequence_with_nominations(seed, n_nodes, n_pods):
    nodes, bound, pods = pf.saturated(seed, n_nodes, n_pods)
    want = _oracle_seq(nodes, bound, pods)
    got = _device_seq(nodes, bound, pods)
    assert got == want
    assert any(w[1] == "nominated" for w in want)
    assert any(w[1] == "scheduled" and w[0] in {x[0] for x in want if x[1] == "nominated"} for w in want)


def test_remove_bound_restores_node_state():
    """kss_remove_bound of every pod on a node leaves that node's columns as if it never held them."""
    nodes, bound, pods = pf.saturated(4, 30, 10)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ctx = _ctx(cc)
    bs = cc.as_boundset()
    ctx.load_bound(bs)
    node0 = [i for i in range(bs.n) if cc.bound["node"][i] == 0]
    assert node0
    ctx.remove_bound(node0)
    g = ctx.node_state()
    assert g["pod_count"][0] == 0
    assert g["requested"][0, 0] == 0 and g["nonzero"][0, 0] == 0
    with pytest.raises(native.KssError):
        ctx.remove_bound(node0[:1])  # no longer in the table
    ctx.close()


def test_window_fixture_cursor():
    """nominated_fixtures.window_fixture on k_schedule: nextStartNodeIndex counts the nominated
    node's status when the search does not reach that node again (the window stops first: 101;
    the node is outside the PreFilterResult list: 1), equal to the C oracle's records."""
    nodes, bound, pods, noms, pct, cursors = nf.window_fixture()
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    idx = {n: i for i, n in enumerate(cc.node_names)}
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    ps = cp.as_struct()
    for n_run, want in ((1, cursors[0]), (2, cursors[1])):
        ch_o, res, st = oracle_c.schedule(prof, cc.as_struct(), ps, n_run, cc.n_nodes, n_classes=len(cc.classes),
                                          n_terms=len(cc.terms), nominations=[(j, idx[n]) for j, n in noms])
        assert st["next_start"] == want
        ctx = _ctx(cc, prof, record=n_run)
        for j, n in noms:
            ctx.nominate(ps, j, idx[n])
        chosen = ctx.schedule_batch(ps, n_run, record=True)
        assert ctx.last_kernel() == "k_schedule"
        np.testing.assert_array_equal(chosen, ch_o)
        assert ctx.next_start_node_index() == want
        for j in range(n_run):
            r = ctx.fetch_record(j)
            np.testing.assert_array_equal(r.fail_plugin[:cc.n_nodes], res.fail_plugin[j, :cc.n_nodes], err_msg=str(j))
            np.testing.assert_array_equal(r.fail_detail[:cc.n_nodes], res.fail_detail[j, :cc.n_nodes], err_msg=str(j))
        ctx.close()


def test_index_keyed_nominations_follow_the_pod():
    """A pod without uid is nominated by its podset index.  The entry belongs to that podset and
    that pod: a call with another podset, or after the pod at that index changed, drops it, so no
    other pod inherits PreferNominatedNode or the nominee self-exclusion; an unchanged podset
    keeps it, and uid-keyed entries survive any podset."""
    nodes, bound, pods, noms, expect = nf.fixture()
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    idx = {n: i for i, n in enumerate(cc.node_names)}
    ps = cp.as_struct()
    ctx = _ctx(cc)
    ctx.nominate(ps, 5, idx["n2"])
    ctx.eval_pod(ps, 0)  # same podset, pod 5 unchanged: kept
    assert ctx.nominations() == [(5, idx["n2"])]
    # another pod list (the pods reversed): "low" now sits at index 5 and must not inherit n2
    cc2, cp2, _ = compile_cluster(nodes, bound, pods[::-1])
    ps2 = cp2.as_struct()
    r = ctx.eval_pod(ps2, 5)
    assert ctx.nominations() == []
    ref = _ctx(cc)
    want = ref.eval_pod(ps2, 5)  # no nominator at all
    assert r.chosen == want.chosen
    np.testing.assert_array_equal(r.fail_plugin[:cc.n_nodes], want.fail_plugin[:cc.n_nodes])
    ref.close()
    # the same podset with the nominated pod edited in place (its priority): dropped
    ctx.nominate(ps, 5, idx["n2"])
    cp.pods["priority"][5] = 7
    ctx.eval_pod(ps, 0)
    assert ctx.nominations() == []
    cp.pods["priority"][5] = 100
    # restaging another list drops it too
    ctx.nominate(ps, 4, idx["n3"])
    ctx.stage(ps2)
    assert ctx.nominations() == []
    # uid-keyed: survives a different podset
    cp.pods["uid"] = 500 + np.arange(cp.n, dtype=np.int32)
    ctx.nominate(ps, 5, idx["n2"])
    ctx.eval_pod(ps2, 0)
    assert ctx.nominations() == [(505, idx["n2"])]
    ctx.close()
