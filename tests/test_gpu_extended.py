"""Extended (scalar) resources on the loop kernels: k_simple and k_spread filter them
(NodeResourcesFit fitsRequest: Insufficient <name>, a zero request skipped) and commit them
(AssumePod adds the pod's request to the node's Requested) in LDS, bit-exact against the C
oracle on fuzzed clusters with one to four extended resources (reference:
simulator/scheduler/config/plugin_test.go:15-36, the default filter set the simulator wraps).
A profile that scores an extended resource keeps the batch on k_schedule."""
import numpy as np
import pytest

import oracle_c
import progfuzz
from kss import abi, native
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu


def _run(prof, nodes, bound, pods, flags=0, kernel=None, shards=None, monkeypatch=None):
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ncl, nt = len(cc.classes), len(cc.terms)
    chosen_o, res, st = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record="meta",
                                          threads=8, n_classes=ncl, n_terms=nt)
    if shards and monkeypatch:
        native.set_option("shards", str(shards))
    ctx = native.Context(prof)
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n, flags=flags)
    if kernel:
        assert ctx.last_kernel() == kernel
    if shards:
        assert ctx.last_geometry()["shards"] == shards
    np.testing.assert_array_equal(chosen, chosen_o)
    meta = ctx.fetch_meta(cp.n)
    for j in range(cp.n):
        m = res.meta(j)
        got = dict(chosen=meta[j, 0], n_feasible=meta[j, 1], scored=meta[j, 2], status=meta[j, 3])
        assert got == {k: m[k] for k in got}, (j, got, m)
        if m["scored"]:
            assert meta[j, 4] == m["best_total"], j
    g = ctx.node_state()
    n = cc.n_nodes
    # every Requested row, the extended resources' included
    np.testing.assert_array_equal(g["requested"][:, :n], st["requested"][:, :n])
    np.testing.assert_array_equal(g["nonzero"][:, :n], st["nonzero"][:, :n])
    np.testing.assert_array_equal(g["pod_count"][:n], st["pod_count"][:n])
    if ncl:
        np.testing.assert_array_equal(g["class_count"][:ncl, :n], st["class_count"][:ncl, :n])
    if nt:
        np.testing.assert_array_equal(g["term_count"][:nt, :n], st["term_count"][:nt, :n])
    ctx.close()
    return cc, res


@pytest.mark.parametrize("seed,n_nodes,n_pods,n_ext", [(11, 80, 300, 1), (12, 400, 400, 2), (13, 1000, 300, 4),
                                                       (14, 5, 60, 3)])
def test_k_simple_extended_resources_match_oracle(seed, n_nodes, n_pods, n_ext):
    nodes, bound, pods = progfuzz.make(seed, n_nodes, n_pods, n_extended=n_ext, programs=False)
    cc, res = _run(abi.default_profile(), nodes, bound, pods, kernel="k_simple")
    assert len(cc.scalars) == n_ext
    # the fuzz does exercise the extended filter: some nodes fail NodeResourcesFit
    assert any(res.meta(j)["n_feasible"] < n_nodes for j in range(len(pods)))


def test_k_simple_extended_resources_forced_shards(monkeypatch):
    nodes, bound, pods = progfuzz.make(15, 333, 250, n_extended=4, programs=False)
    _run(abi.default_profile(), nodes, bound, pods, kernel="k_simple", shards=7, monkeypatch=monkeypatch)


def test_k_simple_extended_resources_custom_profile():
    """k_simple<false> (profile in LDS) with extended resources filtered, not scored."""
    prof = abi.default_profile()
    prof.fit_strategy = abi.KSS_FIT_MOST_ALLOCATED
    prof.fit_weight[0], prof.fit_weight[1] = 2, 3
    prof.weight[abi.KSS_S_TAINT_TOLERATION] = 5
    nodes, bound, pods = progfuzz.make(16, 300, 300, n_extended=3, programs=False)
    _run(prof, nodes, bound, pods, kernel="k_simple")


@pytest.mark.parametrize("seed,n_nodes,n_pods,n_ext", [(21, 60, 200, 1), (22, 300, 300, 4), (23, 700, 250, 2)])
def test_k_spread_extended_resources_match_oracle(seed, n_nodes, n_pods, n_ext):
    nodes, bound, pods = progfuzz.make(seed, n_nodes, n_pods, n_extended=n_ext)
    cc, _ = _run(abi.default_profile(), nodes, bound, pods, kernel="k_spread")
    assert len(cc.scalars) == n_ext


def test_k_spread_extended_resources_forced_shards(monkeypatch):
    nodes, bound, pods = progfuzz.make(24, 211, 150, n_extended=4)
    _run(abi.default_profile(), nodes, bound, pods, kernel="k_spread", shards=9, monkeypatch=monkeypatch)


def test_scored_extended_resource_stays_on_k_schedule():
    """A profile whose LeastAllocated strategy scores an extended resource: k_schedule."""
    nodes, bound, pods = progfuzz.make(25, 120, 120, n_extended=1, programs=False)
    cc, _, _ = compile_cluster(nodes, bound, pods)
    prof = abi.default_profile()
    prof.fit_n = 3
    prof.fit_res[2] = abi.KSS_RES_SCALAR0 + cc.scalars.index(progfuzz.R_GPU)
    prof.fit_weight[2] = 1
    _run(prof, nodes, bound, pods, kernel="k_schedule")
