"""Lazy annotation formatting (csrc/kss_host.cpp) reproduces resultstore.Store.GetStoredResult
(store.go:133-198) byte for byte against the object-level oracle's Go-JSON restatement."""
import json
import os

import numpy as np
import pytest

import k8s_oracle
import oracle_c
from kss import abi, native, synth
from kss.compile import compile_cluster

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "readme_known_answer.json")))


def _format_from_oracle(cc, cp, res, j, prof, pod_aware=False):
    names, keep = native.make_names(cc.node_names, cc.taints, cc.scalars, cp.messages)
    r = native.PodResult(cc.n_nodes)
    r.fail_plugin[:] = res.fail_plugin[j]
    r.fail_detail[:] = res.fail_detail[j]
    r.raw[:] = res.raw[j]
    r.norm[:] = res.norm[j]
    r.total[:] = res.total[j]
    m = res.meta(j)
    r.s.n_feasible, r.s.chosen, r.s.scored, r.s.status = m["n_feasible"], m["chosen"], m["scored"], m["status"]
    if pod_aware:
        return native.format_annotations_ex(names, prof, r, cc.n_nodes, len(cc.taints), len(cc.scalars),
                                            cp.as_struct(), j)
    return native.format_annotations_ex(names, prof, r, cc.n_nodes, len(cc.taints), len(cc.scalars))


@pytest.mark.parametrize("config,n_nodes,n_pods", [(1, 10, 120), (3, 40, 120)])
def test_formatter_matches_object_oracle(config, n_nodes, n_pods):
    nodes, bound, pods = synth.make_cluster(config, n_nodes, n_pods)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    prof = abi.default_profile()
    ch, res, _ = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes,
                                   n_classes=len(cc.classes), n_terms=len(cc.terms))
    o = k8s_oracle.Oracle(nodes, bound)
    kinds = set()
    for j in range(cp.n):
        want = o.annotations(o.schedule_one(pods[j]))
        got = _format_from_oracle(cc, cp, res, j, prof)
        assert got == want, j
        kinds.add((res.meta(j)["scored"], ch[j] >= 0))
    assert (1, True) in kinds


def test_formatter_readme_known_answer():
    cc, cp, _ = compile_cluster(GOLD["nodes"], (), [GOLD["pod"]])
    prof = abi.default_profile()
    ch, res, _ = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), 1, cc.n_nodes)
    got = _format_from_oracle(cc, cp, res, 0, prof)
    for k, v in GOLD["expected"].items():
        if isinstance(v, dict):
            assert json.loads(got[k]) == v, k
        else:
            assert got[k] == v, k


def test_go_json_escaping():
    names, keep = native.make_names(["a<b>&\"c\\", "d\n "], [], [])
    r = native.PodResult(2)
    r.fail_plugin[:] = 1
    r.s.chosen = -1
    r.s.status = 1
    got = native.format_annotations_ex(names, abi.default_profile(), r, 2, 0, 0)
    want = k8s_oracle.go_json({"a<b>&\"c\\": {"NodeUnschedulable": "node(s) were unschedulable"},
                               "d\n ": {"NodeUnschedulable": "node(s) were unschedulable"}})
    assert got["scheduler-simulator/filter-result"] == want
    assert "\\u003c" in want and "\\u2028" in want


@pytest.mark.parametrize("pct", [0, 30])
def test_formatter_window_matches_object_oracle(pct):
    """percentageOfNodesToScore below 100: filter-result lists the visited nodes (the dropped
    one as all-passed), score-result / finalscore-result only the kept ones, and nodes past the
    stop are absent -- the formatter over the C oracle's records equals the object oracle's
    store.go restatement for every pod (pod-aware: the PreFilterResult sets of test_oracle_crosscheck)."""
    from test_oracle_crosscheck import with_name_sets
    nodes, bound, pods = synth.make_cluster(1, 220, 90)
    pods = with_name_sets(pods, [n["metadata"]["name"] for n in nodes], every=4, size=120)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    ch, res, _ = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes)
    o = k8s_oracle.Oracle(nodes, bound, percentage_of_nodes_to_score=pct)
    dropped = 0
    for j in range(cp.n):
        r = o.schedule_one(pods[j])
        dropped += r["dropped"] is not None
        assert _format_from_oracle(cc, cp, res, j, prof, pod_aware=True) == o.annotations(r), j
    assert dropped > 0
