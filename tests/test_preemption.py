"""DefaultPreemption PostFilter dry run: the object-level restatement
(oracle/k8s_preemption.py) against hand-derived expectations (tests/preempt_fixtures.py),
the annotation it produces, and the compiled bound-pod table the device path uses."""
import json

import numpy as np
import pytest

import k8s_oracle as ko
import k8s_preemption as kp
import preempt_fixtures as pf
from kss import abi
from kss.compile import compile_cluster


def test_oracle_matches_hand_derived():
    nodes, bound, pods, expect = pf.fixture()
    o = ko.Oracle(nodes, bound)
    for p, (status, node, victims) in zip(pods, expect):
        r = o.schedule_one(p)
        pre = kp.preempt(o, p, r)
        got_node = ko._name(o.nodes[pre["nominated"]]) if pre["nominated"] is not None else None
        assert (pre["status"], got_node, [v[1] for v in pre["victims"]]) == (status, node, victims), p["metadata"]["name"]


def test_nominated_annotation():
    """store.go:436-456: every node of the status map, the nominated one with
    {"DefaultPreemption": "preemption victim"}."""
    nodes, bound, pods, _ = pf.fixture()
    o, out = kp.schedule_with_preemption(nodes, bound, pods[:1])
    r, pre, ann = out[0]
    post = json.loads(ann["scheduler-simulator/postfilter-result"])
    assert post["a"] == {"DefaultPreemption": kp.NOMINATED_MESSAGE}
    assert post["b"] == {} and set(post) == set(r["filter"])
    assert ann["scheduler-simulator/selected-node"] == ""


def test_prefilter_failure_has_no_candidate():
    nodes, bound, pods, _ = pf.fixture()
    p = pf.pod("conflict", 10, "100m", affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["a"]},
                                               {"key": "metadata.name", "operator": "In", "values": ["b"]}]}]}}})
    o = ko.Oracle(nodes, bound)
    r = o.schedule_one(p)
    assert r["status"] == "prefilter"
    assert kp.preempt(o, p, r)["status"] == "no_candidate"


def test_compiled_bound_table_matches_node_state():
    nodes, bound, pods = pf.saturated(3, 40, 20)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    b = cc.bound
    n = len(cc.bound_names)
    assert n == len(bound)
    np.testing.assert_array_equal(np.bincount(b["node"][:n], minlength=cc.n_nodes), cc.arrays["pod_count"])
    req = np.zeros_like(cc.arrays["requested"])
    for i in range(n):
        req[:, b["node"][i]] += b["req"][:, i]
    np.testing.assert_array_equal(req, cc.arrays["requested"])
    assert set(b["priority"][:n]) <= {0, 10, 100, 1000}
    assert (b["start"][:n] == abi.KSS_START_UNSET).any() and (b["start"][:n] != abi.KSS_START_UNSET).any()
    assert set(int(x) for x in cp.pods["priority"]) <= {0, 10, 100, 1000, 5000}
    never = [bool(p["spec"].get("preemptionPolicy") == "Never") for p in pods]
    assert [bool(f & abi.KSS_POD_PREEMPT_NEVER) for f in cp.pods["flags"]] == never


@pytest.mark.parametrize("seed", [1, 2])
def test_saturated_clusters_nominate(seed):
    """The fuzz generator the GPU parity test uses reaches nominations, FitErrors and
    not-eligible pods."""
    nodes, bound, pods = pf.saturated(seed, 60, 40)
    o, out = kp.schedule_with_preemption(nodes, bound, pods)
    kinds = {pre["status"] for _, pre, _ in out if pre}
    assert "nominated" in kinds and "no_candidate" in kinds


STATUS = {abi.KSS_PREEMPT_NOMINATED: "nominated", abi.KSS_PREEMPT_NO_CANDIDATE: "no_candidate",
          abi.KSS_PREEMPT_NOT_ELIGIBLE: "not_eligible", abi.KSS_PREEMPT_SCHEDULABLE: "schedulable"}


def _c_dry_runs(nodes, bound, pods, threads, nominations=()):
    """The C restatement (oracle/kss_oracle.c kss_oracle_postfilter) of every pod against the
    initial snapshot (nothing committed), as (status, nominated node, victims, criteria).
    nominations: [(pod index, node index)] in the nominator."""
    import oracle_c
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    cl, ps, bs = cc.as_struct(), cp.as_struct(), cc.as_boundset()

    def victim(v):
        return cc.bound_names[v][1]

    out = []
    for j in range(cp.n):
        r = oracle_c.postfilter(abi.default_profile(), cl, ps, j, bs, threads=threads, nominations=nominations)
        nom = cc.node_names[r["nominated"]] if r["nominated"] >= 0 else None
        out.append((STATUS[r["status"]], nom, [victim(v) for v in r["victims"]],
                    (r["n_potential"], r["n_candidates"])))
    return out


def _py_dry_runs(nodes, bound, pods, nominations=()):
    o = ko.Oracle(nodes, bound)
    for a, b in nominations:
        o.nominate(pods[a], b)
    out = []
    for p in pods:
        r = o.schedule_one(p, commit=False)
        pre = kp.preempt(o, p, r)
        nom = ko._name(o.nodes[pre["nominated"]]) if pre["nominated"] is not None else None
        out.append((pre["status"], nom, [v[1] for v in pre["victims"]], (pre["n_potential"], pre["n_candidates"])))
    return out


def test_c_postfilter_matches_hand_derived():
    """The hand-derived fixture, one dry run per pod on the unchanged snapshot."""
    nodes, bound, pods, _ = pf.fixture()
    got = _c_dry_runs(nodes, bound, pods, threads=2)
    want = _py_dry_runs(nodes, bound, pods)
    for j, (g, w) in enumerate(zip(got, want)):
        if w[0] == "schedulable":  # PostFilter never runs for these; a Never pod is refused first
            assert g[0] in ("schedulable", "not_eligible"), j
        else:
            assert g == w, (j, pods[j]["metadata"]["name"])


@pytest.mark.parametrize("seed,n_nodes,n_pods,threads", [(1, 60, 40, 1), (2, 60, 40, 4), (3, 200, 60, 8)])
def test_c_postfilter_matches_object_oracle(seed, n_nodes, n_pods, threads):
    """Saturated clusters: status, nominated node, victims in eviction order and the
    potential / candidate counts equal the object-level restatement, at any thread count."""
    nodes, bound, pods = pf.saturated(seed, n_nodes, n_pods)
    got = _c_dry_runs(nodes, bound, pods, threads)
    want = _py_dry_runs(nodes, bound, pods)
    kinds = set()
    for j, (g, w) in enumerate(zip(got, want)):
        kinds.add(w[0])
        if w[0] == "schedulable":  # PostFilter never runs for these; a Never pod is refused first
            assert g[0] in ("schedulable", "not_eligible"), j
        else:
            assert g == w, j
    assert "nominated" in kinds


@pytest.mark.parametrize("seed,n_nodes,n_pods,threads", [(1, 60, 40, 2), (3, 200, 60, 8), (5, 80, 60, 4)])
def test_c_postfilter_with_nominees_matches_object_oracle(seed, n_nodes, n_pods, threads):
    """The same dry runs with a nominator of a dozen pods on random nodes: the nominees of equal or
    higher priority take part in every filter call (the statuses and SelectVictimsOnNode)."""
    import random
    nodes, bound, pods = pf.saturated(seed, n_nodes, n_pods)
    rnd = random.Random(seed)
    noms = [(j, rnd.randrange(n_nodes)) for j in rnd.sample(range(n_pods), 12)]
    got = _c_dry_runs(nodes, bound, pods, threads, noms)
    want = _py_dry_runs(nodes, bound, pods, noms)
    plain = _py_dry_runs(nodes, bound, pods)
    for j, (g, w) in enumerate(zip(got, want)):
        if w[0] == "schedulable":
            assert g[0] in ("schedulable", "not_eligible"), j
        else:
            assert g == w, j
    assert want != plain  # the nominees changed some dry run
