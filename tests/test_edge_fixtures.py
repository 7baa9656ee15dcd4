"""Both oracles (and the lazy annotation formatter) against hand-derived expectations for
every filter reason string and branch (tests/edge_fixtures.py): NodeUnschedulable with and
without the toleration, NodeName, NoSchedule / NoExecute / PreferNoSchedule taints,
In / NotIn / Exists / DoesNotExist / Gt / Lt, nodeSelector, matchFields metadata.name
(PreFilterResult, union, open term, conflict), Too many pods, cpu / memory /
ephemeral-storage / extended-resource shortfalls and their joined message, init-container
requests, the PodTopologySpread missing-label and skew reasons, system-defaulted spreading
with a zone-less node, the three InterPodAffinity reasons and a non-identity nodeTree order.
"""
import pytest

import edge_fixtures as ef
import k8s_oracle
from crosscheck import run_both
from kss import abi
from kss.compile import compile_cluster
from test_format import _format_from_oracle

PTS = abi.KSS_S_POD_TOPOLOGY_SPREAD


@pytest.mark.parametrize("name", sorted(ef.FIXTURES))
def test_object_oracle_matches_hand_derived(name):
    nodes, bound, pods, expect = ef.FIXTURES[name]()
    o = k8s_oracle.Oracle(nodes, bound)
    names = [k8s_oracle._name(n) for n in o.nodes]
    for j, (p, exp) in enumerate(zip(pods, expect)):
        r = o.schedule_one(p)
        pts = None
        if r["scored"]:
            pts = {names[i]: (r["raw"]["PodTopologySpread"][i], r["norm"]["PodTopologySpread"][i])
                   for i in r["raw"]["PodTopologySpread"]}
        ef.check_expect(o.annotations(r), exp, pts, where=(name, j))


@pytest.mark.parametrize("name", sorted(ef.FIXTURES))
def test_c_oracle_and_formatter_match_hand_derived(name):
    nodes, bound, pods, expect = ef.FIXTURES[name]()
    cc, cp, chosen, res = run_both(nodes, bound, pods)  # the two oracles agree first
    prof = abi.default_profile()
    o = k8s_oracle.Oracle(nodes, bound)
    for j, exp in enumerate(expect):
        ann = _format_from_oracle(cc, cp, res, j, prof, pod_aware=True)
        assert ann == o.annotations(o.schedule_one(pods[j])), (name, j)  # all 13 values, byte for byte
        pts = {nm: (int(res.raw[j, PTS, i]), int(res.norm[j, PTS, i])) for i, nm in enumerate(cc.node_names)}
        ef.check_expect(ann, exp, pts if res.meta(j)["scored"] else None, where=(name, j))


def test_node_tree_order_is_canonical_order():
    nodes, bound, pods, _ = ef.fx_node_tree_order()
    cc, _, _ = compile_cluster(nodes, bound, pods)
    assert cc.node_names == ef.TREE_ORDER
    assert [k8s_oracle._name(n) for n in k8s_oracle.Oracle(nodes, bound).nodes] == ef.TREE_ORDER


def test_every_filter_reason_is_covered():
    """The fixtures together exercise every reason string the filter plugins emit."""
    seen = set()
    for fx in ef.FIXTURES.values():
        for exp in fx()[3]:
            for f in exp["filter"].values():
                if f is not None:
                    seen.add(f[1])
    for msg in (ef.M_UNSCHED, ef.M_NAME, ef.M_AFF, ef.M_PTS, ef.M_PTS_LABEL, ef.M_IPA_AFF, ef.M_IPA_ANTI,
                ef.M_IPA_EXIST, "Too many pods", "Insufficient cpu", "Insufficient memory",
                "Insufficient ephemeral-storage", "Insufficient example.com/gpu", ef.M_PORTS):
        assert msg in seen, msg
    assert any(m.startswith("node(s) had untolerated taint") for m in seen)
