"""v1.26 PodTopologySpread with several constraints on one topology key — hand-derived.

calPreFilterState (pkg/scheduler/framework/plugins/podtopologyspread/filtering.go, v1.26)
keys TpPairToMatchNum by topology pair and, per node, sets tpCounts[pair] = count for each
admitting constraint in order, so the LAST constraint on a key decides the node's count;
the critical path (global minimum) is per key.  initPreScoreState / PreScore (scoring.go)
share one counter per pair across the constraints on a key, and every pair counts in the
topoSize of the first constraint on the key (the later ones weigh log(0 + 2)).

Cluster: zone z1 = {n1, n2}, zone z2 = {n3, n4}; bound pods n1: 2 x app=a, n2: 1 x app=b,
n3: 4 x app=b.  Pending (both labelled app=c, so neither selector matches them):

  P1: DoNotSchedule zone/app=a and DoNotSchedule zone/app=b, maxSkew 1.
      Per node the app=b count wins: TpPairToMatchNum z1 = 0 + 1 = 1, z2 = 4 + 0 = 4,
      minimum 1.  z1: 1 - 1 = 0 <= 1 passes; z2: 4 - 1 = 3 > 1 fails.  (Per-constraint
      counting would fail every node: app=a z1 = 2 against a minimum of 0.)
  P2: ScheduleAnyway zone/app=a maxSkew 1 and ScheduleAnyway zone/app=b maxSkew 2.
      Pair counters: z1 = (2 + 0) + (0 + 1) = 3, z2 = 0 + 4 = 4; topoSize 2 for the first,
      0 for the second: weights log(4), log(2).  Raw score
      cnt * log 4 + 0 + cnt * log 2 + 1: z1 round(3 log 4 + 3 log 2 + 1) = 7, z2
      round(4 log 4 + 4 log 2 + 1) = 9.  (Per-constraint counting gives 5 and 7.)
"""
import math

import numpy as np

from crosscheck import run_both
from kss import abi

ZONE = "topology.kubernetes.io/zone"


def _node(name, zone):
    return {"metadata": {"name": name, "labels": {"kubernetes.io/hostname": name, ZONE: zone}},
            "spec": {}, "status": {"allocatable": {"cpu": "8", "memory": "32Gi", "pods": "110"}}}


def _bound(name, node, app):
    return {"metadata": {"name": name, "namespace": "default", "labels": {"app": app}},
            "spec": {"nodeName": node, "containers": [{"name": "c", "resources": {"requests": {"cpu": "100m"}}}]}}


def _pending(name, when, skews):
    cons = [{"maxSkew": skews[0], "topologyKey": ZONE, "whenUnsatisfiable": when,
             "labelSelector": {"matchLabels": {"app": "a"}}},
            {"maxSkew": skews[1], "topologyKey": ZONE, "whenUnsatisfiable": when,
             "labelSelector": {"matchLabels": {"app": "b"}}}]
    return {"metadata": {"name": name, "namespace": "default", "labels": {"app": "c"}},
            "spec": {"containers": [{"name": "c", "resources": {"requests": {"cpu": "100m"}}}],
                     "topologySpreadConstraints": cons}}


def fixture():
    nodes = [_node("n1", "z1"), _node("n2", "z1"), _node("n3", "z2"), _node("n4", "z2")]
    bound = [_bound("a1", "n1", "a"), _bound("a2", "n1", "a"), _bound("b1", "n2", "b")]
    bound += [_bound(f"b{i}", "n3", "b") for i in range(2, 6)]
    pods = [_pending("p1", "DoNotSchedule", (1, 1)), _pending("p2", "ScheduleAnyway", (1, 2))]
    return nodes, bound, pods


def go_log(x):
    return math.log(x)  # the rounded results below do not depend on the last bits of the logarithm


def test_same_key_constraints_both_oracles():
    cc, cp, chosen, res = run_both(*fixture())  # object-level and SoA-level oracles agree
    idx = {nm: i for i, nm in enumerate(cc.node_names)}
    pts = abi.FILTER_PLUGINS.index("PodTopologySpread")
    fp = res.fail_plugin[0]
    assert [int(fp[idx[n]]) for n in ("n1", "n2", "n3", "n4")] == [0, 0, pts, pts]
    assert res.meta(0)["n_feasible"] == 2
    raw = res.raw[1][abi.KSS_S_POD_TOPOLOGY_SPREAD]
    want = {"z1": round(3 * go_log(4) + 3 * go_log(2) + 1), "z2": round(4 * go_log(4) + 4 * go_log(2) + 1)}
    assert (want["z1"], want["z2"]) == (7, 9)
    for n, z in (("n1", "z1"), ("n2", "z1"), ("n3", "z2"), ("n4", "z2")):
        assert int(raw[idx[n]]) == want[z], (n, int(raw[idx[n]]))
    assert np.all(chosen >= 0)
