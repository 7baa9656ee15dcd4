"""percentageOfNodesToScore < 100 on k_spread (kss_spread.cuh spread_schedule WIN): the
findNodesThatPassFilters window in its Parallelism = 1 order, for batches with PodTopologySpread /
InterPodAffinity programs, against the C oracle (which filters every node and cuts the list
afterwards, kss_oracle.c).  Chosen nodes, per-pod outcomes (n_feasible = the kept nodes), the
final node and count state, and nextStartNodeIndex.

  * the C3 recipe at 5,000 nodes (K = 500 adaptive, 1,500 at 30 %) on the XCD-local grid (32
    shards), unrestricted, on 24 shards, and across chunk launches (the cursor handed on through
    the device word), from a set cursor, two runs each;
  * C4's recipe at 20,000 nodes (448-lane shards, the 512-lane kernel; more than 64 shards: the
    two-level selectHost exchange);
  * program fuzz (every constraint / term kind; PreScore sizes and IgnoredNodes over the kept
    nodes) on 2 / 9 shards and the 101-node edge (K = 100);
  * a custom profile keeps the window on k_schedule, with the same results.
"""
import os

import numpy as np
import pytest

import oracle_c
import progfuzz
from kss import abi, native
from kss.compile import compile_cluster
from kss.synth import SEED_BASE

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _prof(pct):
    p = abi.default_profile()
    p.pct_nodes_to_score = pct
    return p


def _check(ctx, chosen, ch_o, res, st, n, N, ncl, nt):
    np.testing.assert_array_equal(chosen, ch_o)
    meta = ctx.fetch_meta(n)
    for j in range(n):
        m = res.meta(j)
        got = dict(chosen=meta[j, 0], n_feasible=meta[j, 1], scored=meta[j, 2], status=meta[j, 3])
        assert got == {k: m[k] for k in got}, (j, got, m)
        if m["scored"]:
            assert meta[j, 4] == m["best_total"], j
    assert ctx.next_start_node_index() == st["next_start"]
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :N], st["requested"][:, :N])
    np.testing.assert_array_equal(g["pod_count"][:N], st["pod_count"][:N])
    if ncl:
        np.testing.assert_array_equal(g["class_count"][:ncl], st["class_count"][:ncl])
    if nt:
        np.testing.assert_array_equal(g["term_count"][:nt], st["term_count"][:nt])


@pytest.mark.parametrize("geometry", ["xcd_local", "unrestricted", "few_shards", "chunks"])
@pytest.mark.parametrize("pct", [0, 30])
def test_c3_window_geometries(pct, geometry):
    n_nodes = 3000 if geometry == "few_shards" else 5000
    n_pods, cursor = 800, 2321
    prof = _prof(pct)
    s = native.Synth(3, SEED_BASE + 3, n_nodes, n_pods)
    ncl, nt = s.cluster.n_classes, s.cluster.n_terms
    ch_o, res, st = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record="meta", threads=THREADS,
                                      n_classes=ncl, n_terms=nt, cursor=cursor)
    if geometry == "unrestricted":
        native.set_option("xcd", 0)
    elif geometry == "few_shards":
        native.set_option("shards", 24)
    elif geometry == "chunks":
        native.set_option("static_bytes", 4 * n_nodes * 150)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    for rep in range(2):
        ctx.reset()
        ctx.set_next_start_node_index(cursor)
        chosen = ctx.run_staged(n_pods)
        assert ctx.last_kernel() == "k_spread", rep
        if geometry == "few_shards":
            assert ctx.last_geometry()["shards"] == 24
        if geometry == "chunks":
            assert ctx.last_timing()[1] >= 2 * 5
        _check(ctx, chosen, ch_o, res, st, n_pods, n_nodes, ncl, nt)
    ctx.close()


def test_c4_recipe_window():
    """C4's recipe (zone DoNotSchedule) at 20,000 nodes, pct 0 (K = 1,000): more than 64 shards of
    448 lanes."""
    n_nodes, n_pods = 20000, 300
    prof = _prof(0)
    s = native.Synth(4, SEED_BASE + 4, n_nodes, n_pods)
    ncl, nt = s.cluster.n_classes, s.cluster.n_terms
    ch_o, res, st = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record="meta", threads=THREADS,
                                      n_classes=ncl, n_terms=nt)
    native.set_option("shards", 80)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    assert ctx.last_kernel() == "k_spread" and ctx.last_geometry()["shards"] == 80
    _check(ctx, chosen, ch_o, res, st, n_pods, n_nodes, ncl, nt)
    ctx.close()


def _no_name_lists(pods):
    """matchFields metadata.name In (a PreFilterResult node list: the window then takes k_schedule)
    turned into NotIn, so the fuzz batch stays on k_spread."""
    for p in pods:
        na = p.get("spec", {}).get("affinity", {}).get("nodeAffinity", {})
        for t in na.get("requiredDuringSchedulingIgnoredDuringExecution", {}).get("nodeSelectorTerms", []):
            for f in t.get("matchFields", []):
                if f.get("key") == "metadata.name" and f.get("operator") == "In":
                    f["operator"] = "NotIn"
    return pods


@pytest.mark.parametrize("shards", [2, 9])
@pytest.mark.parametrize("pct", [0, 40])
def test_program_fuzz_window(shards, pct):
    prof = _prof(pct)
    on_spread = 0
    for seed in (20, 21, 22, 51):
        nodes, bound, pods = progfuzz.make(seed, 211, 150)
        pods = _no_name_lists(pods)
        cc, cp, _ = compile_cluster(nodes, bound, pods)
        ncl, nt = len(cc.classes), len(cc.terms)
        ch_o, res, st = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record="meta",
                                          threads=THREADS, n_classes=ncl, n_terms=nt, cursor=57)
        native.set_option("shards", shards)
        ctx = native.Context(prof)
        ctx.load(cc.as_struct())
        ctx.set_next_start_node_index(57)
        chosen = ctx.schedule_batch(cp.as_struct(), cp.n)
        on_spread += ctx.last_kernel() == "k_spread"
        _check(ctx, chosen, ch_o, res, st, cp.n, cc.n_nodes, ncl, nt)
        ctx.close()
    assert on_spread >= 3


@pytest.mark.parametrize("n_nodes", [101, 180])
def test_spread_window_edges(n_nodes):
    prof = _prof(0)
    n_pods = 400
    s = native.Synth(3, SEED_BASE + 3, n_nodes, n_pods)
    ncl, nt = s.cluster.n_classes, s.cluster.n_terms
    ch_o, res, st = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record="meta", threads=THREADS,
                                      n_classes=ncl, n_terms=nt)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    assert ctx.last_kernel() == "k_spread"
    _check(ctx, chosen, ch_o, res, st, n_pods, n_nodes, ncl, nt)
    ctx.close()


def test_custom_profile_window_on_k_schedule():
    prof = _prof(0)
    prof.weight[abi.KSS_S_TAINT_TOLERATION] = 5
    n_nodes, n_pods = 1500, 200
    s = native.Synth(3, SEED_BASE + 3, n_nodes, n_pods)
    ncl, nt = s.cluster.n_classes, s.cluster.n_terms
    ch_o, res, st = oracle_c.schedule(prof, s.cluster, s.pods, n_pods, n_nodes, record="meta", threads=THREADS,
                                      n_classes=ncl, n_terms=nt)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(n_pods)
    assert ctx.last_kernel() == "k_schedule"
    _check(ctx, chosen, ch_o, res, st, n_pods, n_nodes, ncl, nt)
    ctx.close()
