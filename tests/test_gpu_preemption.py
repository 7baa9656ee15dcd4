"""DefaultPreemption PostFilter dry run on the device (k_preempt through kss_postfilter_pod)
against the object-level restatement (oracle/k8s_preemption.py): status, nominated node and
the victims in eviction order for every unschedulable pod of a sequence -- the hand-derived
fixture and seeded saturated clusters (every node nearly full of pods of mixed priority),
with the pods placed earlier in the sequence (per-pod commits or a batch) as potential
victims."""
import pytest

import k8s_oracle as ko
import k8s_preemption as kp
import preempt_fixtures as pf
from kss import abi, native
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu

STATUS = {abi.KSS_PREEMPT_NOMINATED: "nominated", abi.KSS_PREEMPT_NO_CANDIDATE: "no_candidate",
          abi.KSS_PREEMPT_NOT_ELIGIBLE: "not_eligible", abi.KSS_PREEMPT_SCHEDULABLE: "schedulable"}


def _oracle(nodes, bound, pods):
    o, out = kp.schedule_with_preemption(nodes, bound, pods)
    res = []
    for r, pre, _ in out:
        if r["selected"] is not None:
            res.append(("scheduled", ko._name(o.nodes[r["selected"]]), []))
        else:
            nom = ko._name(o.nodes[pre["nominated"]]) if pre["nominated"] is not None else None
            res.append((pre["status"], nom, [v[1] for v in pre["victims"]]))
    return res


def _device(nodes, bound, pods, batch_first=0):
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ps = cp.as_struct()
    ctx = native.Context(abi.default_profile(), max_pods_record=max(batch_first, 1))
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    bs = cc.as_boundset()
    ctx.load_bound(bs)

    def victim_name(v):
        return cc.bound_names[v][1] if v >= 0 else cp.names[-1 - v][1]

    out = []
    if batch_first:
        chosen = ctx.schedule_batch(ps, batch_first, record=True)
        for j in range(batch_first):
            if chosen[j] >= 0:
                out.append(("scheduled", cc.node_names[chosen[j]], []))
            else:
                out.append(None)  # the oracle's dry run of these is checked per pod below
    for j in range(batch_first, cp.n):
        r = ctx.eval_pod(ps, j)
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
            out.append(("scheduled", cc.node_names[r.chosen], []))
            continue
        pre = ctx.postfilter_pod(ps, j)
        assert pre["n_victims"] == len(pre["victims"])
        nom = cc.node_names[pre["nominated"]] if pre["nominated"] >= 0 else None
        out.append((STATUS[pre["status"]], nom, [victim_name(v) for v in pre["victims"]]))
    ctx.close()
    return out


def test_hand_derived_fixture_on_device():
    nodes, bound, pods, expect = pf.fixture()
    assert _device(nodes, bound, pods) == [tuple(e) for e in expect]


@pytest.mark.parametrize("seed,n_nodes,n_pods", [(1, 60, 40), (2, 60, 40), (3, 200, 60), (4, 500, 60)])
def test_saturated_sequence_matches_oracle(seed, n_nodes, n_pods):
    nodes, bound, pods = pf.saturated(seed, n_nodes, n_pods)
    want = _oracle(nodes, bound, pods)
    got = _device(nodes, bound, pods)
    assert got == want
    assert any(w[0] == "nominated" for w in want)


def test_batch_commits_become_victims():
    """Pods placed by a device batch are in the bound table of the next dry runs."""
    nodes, bound, pods = pf.saturated(5, 80, 60)
    want = _oracle(nodes, bound, pods)
    got = _device(nodes, bound, pods, batch_first=30)
    for j, (g, w) in enumerate(zip(got, want)):
        if g is None:
            assert w[0] != "scheduled", j
        else:
            assert g == w, j
