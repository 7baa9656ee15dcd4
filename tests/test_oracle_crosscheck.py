"""The SoA-level C oracle agrees with the object-level Python oracle on seeded synthetic clusters."""
import pytest

from crosscheck import run_both
from kss import synth


@pytest.mark.parametrize("config,n_nodes,n_pods", [(1, 100, 300), (1, 12, 200), (5, 40, 120)])
def test_default_profile(config, n_nodes, n_pods):
    nodes, bound, pods = synth.make_cluster(config, n_nodes, n_pods)
    run_both(nodes, bound, pods)


@pytest.mark.parametrize("n_nodes,n_pods", [(30, 150), (90, 200)])
def test_spread_and_interpod_affinity(n_nodes, n_pods):
    nodes, bound, pods = synth.make_cluster(3, n_nodes, n_pods)
    run_both(nodes, bound, pods)


def test_zone_spread_c4_recipe():
    nodes, bound, pods = synth.make_cluster(4, 60, 150)
    run_both(nodes, bound, pods)


@pytest.mark.parametrize("seed", range(8))
def test_program_fuzz(seed):
    """Every spread / inter-pod program kind (tests/progfuzz.py), the programs k_spread's
    GPU parity tests run, with per-node verdicts and raw / normalized scores compared."""
    import progfuzz
    nodes, bound, pods = progfuzz.make(1000 + seed, 70, 110)
    run_both(nodes, bound, pods)


# ---- percentageOfNodesToScore below 100 (numFeasibleNodesToFind / nextStartNodeIndex) ----

def with_name_sets(pods, node_names, every=4, size=120, seed=7):
    """Every `every`-th pod gains a required node affinity term whose matchFields metadata.name
    In lists `size` node names: NodeAffinity's PreFilterResult, so findNodesThatPassFilters
    walks that set (size >= 100: the window applies inside it)."""
    import copy
    import random
    rnd = random.Random(seed)
    out = []
    for j, p in enumerate(pods):
        p = copy.deepcopy(p)
        if j % every == 0:
            names = rnd.sample(node_names, min(size, len(node_names)))
            aff = p["spec"].setdefault("affinity", {})
            aff["nodeAffinity"] = dict(aff.get("nodeAffinity") or {}, requiredDuringSchedulingIgnoredDuringExecution={
                "nodeSelectorTerms": [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": names}]}]})
        out.append(p)
    return out


@pytest.mark.parametrize("pct", [0, 30, 50, 99])
@pytest.mark.parametrize("config,n_nodes,n_pods", [(1, 250, 160), (1, 101, 120), (1, 100, 80)])
def test_window_default_profile(pct, config, n_nodes, n_pods):
    """Default profile with the window: the C oracle (filter every node, then cut the list) and
    the object oracle (visit nodes one at a time, stop) agree on verdicts, the dropped node,
    scores over the kept nodes and the chosen node; 100 nodes is the minFeasibleNodesToFind edge
    (every node kept), 101 the first size where the search stops early."""
    nodes, bound, pods = synth.make_cluster(config, n_nodes, n_pods)
    run_both(nodes, bound, pods, pct=pct)


@pytest.mark.parametrize("pct", [0, 40])
def test_window_spread_and_interpod(pct):
    """PodTopologySpread's PreScore sizes and InterPodAffinity's normalisation over the kept
    nodes only (config-3 programs on 180 nodes)."""
    nodes, bound, pods = synth.make_cluster(3, 180, 140)
    run_both(nodes, bound, pods, pct=pct)


def test_window_prefilter_result_sets():
    """PreFilterResult sets of 120 nodes: the window walks the set in canonical order from
    nextStartNodeIndex modulo the set size, and a short set (every node kept) still folds the
    index modulo its size."""
    nodes, bound, pods = synth.make_cluster(1, 200, 160)
    names = [n["metadata"]["name"] for n in nodes]
    pods = with_name_sets(pods, names, every=3, size=120)
    pods = with_name_sets(pods, names, every=7, size=30, seed=11)
    run_both(nodes, bound, pods, pct=20)


def test_num_feasible_nodes_to_find_table():
    """numFeasibleNodesToFind (v1.26): the adaptive percentage and both floors."""
    import k8s_oracle
    f = k8s_oracle.num_feasible_nodes_to_find
    assert [f(n, 0) for n in (50, 99, 100, 101, 200, 1000, 5000, 100000)] == [50, 99, 100, 100, 100, 420, 500, 5000]
    assert f(5000, 100) == 5000 and f(5000, 30) == 1500 and f(300, 10) == 100 and f(6000, 1) == 100
