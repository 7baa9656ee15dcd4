"""Snapshot I/O (kss/snapshot.py): ResourcesForSnap JSON <-> objects <-> compiled SoA, the
scheduler configuration -> kss_profile mapping (the simulator's mergePluginSet and weight
rules), and the delta computation of the generation sync."""
import json

import numpy as np
import pytest

from kss import abi, snapshot, synth
from kss.compile import Unsupported, compile_cluster


def _same_profile(a, b):
    return bytes(a) == bytes(b)


def test_round_trip_compiles_identically():
    nodes, bound, pods = synth.make_cluster(3, n_nodes=60, n_pods=40)
    doc = json.dumps(synth.to_resources_for_snap(nodes, bound, pods))
    snap = snapshot.read_snapshot(doc)
    assert len(snap.bound) == len(bound) and len(snap.pending) == len(pods)
    cc0, cp0, _ = compile_cluster(nodes, bound, pods)
    cc1, cp1, _ = compile_cluster(snap.nodes, snap.bound, snap.pending, snap.namespaces)
    for k, v in cc0.arrays.items():
        np.testing.assert_array_equal(cc1.arrays[k], v, err_msg=k)
    assert cp0.pods.tobytes() == cp1.pods.tobytes()
    again = snapshot.read_snapshot(snapshot.write_snapshot(snap))
    assert again.bound == snap.bound and again.pending == snap.pending and again.nodes == snap.nodes


def test_priority_class_resolution():
    doc = {"nodes": [], "namespaces": [],
           "priorityClasses": [{"metadata": {"name": "high"}, "value": 1000},
                               {"metadata": {"name": "base"}, "value": 7, "globalDefault": True}],
           "pods": [{"metadata": {"name": "a"}, "spec": {"priorityClassName": "high"}},
                    {"metadata": {"name": "b"}, "spec": {}},
                    {"metadata": {"name": "c"}, "spec": {"priority": 3, "priorityClassName": "high"}}]}
    snap = snapshot.read_snapshot(doc)
    assert [p["spec"].get("priority") for p in snap.pending] == [1000, 7, 3]


def test_default_config_is_the_default_profile():
    d = abi.default_profile()
    d.pct_nodes_to_score = 0  # the simulator's scheduler always runs with the v1 default: adaptive
    assert _same_profile(snapshot.profile_from_config(None), d)
    assert _same_profile(snapshot.profile_from_config({"profiles": [{"schedulerName": "default-scheduler"}]}), d)
    # the north_star / bench workloads opt in to scoring every node
    assert _same_profile(snapshot.profile_from_config(None, pct_nodes_to_score=100), abi.default_profile())


def test_config_weights_disables_and_args():
    cfg = {"profiles": [{
        "plugins": {"multiPoint": {"enabled": [{"name": "NodeResourcesFit", "weight": 5},
                                               {"name": "ImageLocality", "weight": 0}]},
                    "score": {"disabled": [{"name": "NodeResourcesBalancedAllocation"}]},
                    "filter": {"disabled": [{"name": "NodePorts"}]}},
        "pluginConfig": [
            {"name": "NodeResourcesFit", "args": {"scoringStrategy": {
                "type": "MostAllocated", "resources": [{"name": "cpu", "weight": 3}, {"name": "memory", "weight": 2}]}}},
            {"name": "InterPodAffinity", "args": {"hardPodAffinityWeight": 4}},
            {"name": "PodTopologySpread", "args": {"defaultingType": "List"}}]}]}
    p = snapshot.profile_from_config(cfg)
    assert p.weight[abi.KSS_S_NODE_RESOURCES_FIT] == 5
    assert p.weight[abi.KSS_S_IMAGE_LOCALITY] == 1  # weight 0 -> 1 (plugins.go:296-300)
    assert not (p.score_enabled >> abi.KSS_S_BALANCED_ALLOCATION) & 1
    assert not (p.filter_enabled >> abi.KSS_F_NODE_PORTS) & 1
    assert (p.filter_enabled >> abi.KSS_F_NODE_RESOURCES_FIT) & 1
    assert p.fit_strategy == abi.KSS_FIT_MOST_ALLOCATED and list(p.fit_weight[:2]) == [3, 2]
    assert p.hard_pod_affinity_weight == 4 and p.system_defaulted == 0


def test_conflicting_weights_framework_vs_store():
    """A plugin weighted differently at Score and MultiPoint: the framework schedules with the
    Score entry's weight; the simulator's store (getScorePluginWeight, plugins.go:288-303:
    Score.Enabled, then the merged MultiPoint, last assignment wins) records finalscores with
    the MultiPoint weight -- an in-tree default when the user's MultiPoint does not list it."""
    cfg = {"profiles": [{"plugins": {
        "score": {"enabled": [{"name": "TaintToleration", "weight": 10}, {"name": "NodeAffinity", "weight": 9}]},
        "multiPoint": {"enabled": [{"name": "NodeAffinity", "weight": 4}]}}}]}
    p = snapshot.profile_from_config(cfg)
    assert p.weight[abi.KSS_S_TAINT_TOLERATION] == 10 and p.weight[abi.KSS_S_NODE_AFFINITY] == 9
    w = snapshot.store_weights_from_config(cfg)
    assert w["TaintToleration"] == 3 and w["NodeAffinity"] == 4 and w["ImageLocality"] == 1
    ps = snapshot.store_profile_from_config(cfg)
    assert ps.weight[abi.KSS_S_TAINT_TOLERATION] == 3 and ps.weight[abi.KSS_S_NODE_AFFINITY] == 4
    assert ps.weight[abi.KSS_S_NODE_RESOURCES_FIT] == 1 and ps.score_enabled == p.score_enabled
    # no conflict: the two agree
    assert snapshot.store_weights_from_config(None)["TaintToleration"] == 3


def test_config_star_disable_and_refusals():
    cfg = {"profiles": [{"plugins": {"multiPoint": {"disabled": [{"name": "*"}],
                                                    "enabled": [{"name": "NodeResourcesFit"},
                                                                {"name": "TaintToleration", "weight": 7}]}}}]}
    p = snapshot.profile_from_config(cfg)
    assert p.filter_enabled == (1 << abi.KSS_F_NODE_RESOURCES_FIT) | (1 << abi.KSS_F_TAINT_TOLERATION)
    assert p.score_enabled == (1 << abi.KSS_S_NODE_RESOURCES_FIT) | (1 << abi.KSS_S_TAINT_TOLERATION)
    assert p.weight[abi.KSS_S_TAINT_TOLERATION] == 7 and p.weight[abi.KSS_S_NODE_RESOURCES_FIT] == 1
    # filterOutNonAllowedChangesOnCfg (simulator/scheduler/scheduler.go:258-275) resets the field
    # to the v1 default 0 whatever the configuration says; 100 only by an explicit opt-in
    assert snapshot.profile_from_config({"percentageOfNodesToScore": 50, "profiles": [{}]}).pct_nodes_to_score == 0
    assert snapshot.profile_from_config({"percentageOfNodesToScore": 100, "profiles": [{}]}).pct_nodes_to_score == 0
    assert snapshot.profile_from_config({"profiles": [{}]}).pct_nodes_to_score == 0
    assert snapshot.profile_from_config(None).pct_nodes_to_score == 0
    assert snapshot.profile_from_config({"profiles": [{}]}, pct_nodes_to_score=30).pct_nodes_to_score == 30
    with pytest.raises(Unsupported):
        snapshot.profile_from_config(None, pct_nodes_to_score=-1)
    with pytest.raises(Unsupported):
        snapshot.profile_from_config({"percentageOfNodesToScore": 101, "profiles": [{}]})
    with pytest.raises(Unsupported):
        snapshot.profile_from_config({"profiles": [{"pluginConfig": [{"name": "NodeResourcesFit", "args": {
            "scoringStrategy": {"type": "RequestedToCapacityRatio"}}}]}]})
    with pytest.raises(Unsupported):
        snapshot.profile_from_config({"profiles": [{"plugins": {"multiPoint": {"enabled": [{"name": "MyPlugin"}]}}}]})


class _Recorder:
    def __init__(self):
        self.calls = []

    def apply_node_delta(self, idx, req, nz, pc):
        self.calls.append(("node", np.array(idx), np.array(req), np.array(pc)))

    def apply_count_delta(self, node, row, val):
        self.calls.append(("count", list(node), list(row), list(val)))

    def apply_port_delta(self, idx, used):
        self.calls.append(("port", np.array(idx), np.array(used)))


def test_delta_rows_are_the_changed_nodes():
    nodes, bound, pods = synth.make_cluster(3, n_nodes=40, n_pods=30)
    later = [dict(p, spec=dict(p["spec"], nodeName=nodes[i % 7]["metadata"]["name"])) for i, p in enumerate(pods[:10])]
    cc0, _, _ = compile_cluster(nodes, bound, pods)
    cc1, _, _ = compile_cluster(nodes, bound + later, pods[10:])
    rec = _Recorder()
    out = snapshot.sync_deltas(rec, cc0, cc1)
    touched = sorted({cc1.node_names.index(nodes[i % 7]["metadata"]["name"]) for i in range(10)})
    assert out["rows"] == len(touched)
    assert sorted(rec.calls[0][1].tolist()) == touched
    assert out["count_cells"] > 0
