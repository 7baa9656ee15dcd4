"""k_spread (kss_spread.cuh): the sequential loop for batches with PodTopologySpread /
InterPodAffinity programs, bit-exact against the C oracle.

  * seeded program fuzz (tests/progfuzz.py: every constraint / term kind, policies,
    unique and shared keys, missing labels) in the automatic, single-workgroup and forced
    multi-shard geometries;
  * several launches per batch (static-word chunks; the count rows the launches commit
    are carried in HBM between them), a non-default profile (k_spread<false>);
  * the device restatement of Go math.Log against the host port, bit for bit;
  * k_spread and k_schedule agree on the same batch.
The full-size C3 / C4 batches are in test_gpu_scale.py.
"""
import numpy as np
import pytest

import oracle_c
import progfuzz
from kss import abi, native
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu

MODES = {"auto": 0, "single": abi.KSS_SCHED_FORCE_SINGLE_WG, "multi": abi.KSS_SCHED_FORCE_MULTI_WG}


def _oracle(prof, cl, ps, n, n_nodes, n_classes, n_terms):
    return oracle_c.schedule(prof, cl, ps, n, n_nodes, record="meta", threads=8, n_classes=n_classes, n_terms=n_terms)


def _check(ctx, res, st, chosen, chosen_o, n, n_nodes, n_classes, n_terms):
    np.testing.assert_array_equal(chosen, chosen_o)
    meta = ctx.fetch_meta(n)
    for j in range(n):
        m = res.meta(j)
        got = dict(chosen=meta[j, 0], n_feasible=meta[j, 1], scored=meta[j, 2], status=meta[j, 3])
        assert got == {k: m[k] for k in got}, (j, got, m)
        if m["scored"]:
            assert meta[j, 4] == m["best_total"], j
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :n_nodes], st["requested"][:, :n_nodes])
    np.testing.assert_array_equal(g["nonzero"][:, :n_nodes], st["nonzero"][:, :n_nodes])
    np.testing.assert_array_equal(g["pod_count"][:n_nodes], st["pod_count"][:n_nodes])
    if n_classes:
        np.testing.assert_array_equal(g["class_count"][:n_classes], st["class_count"][:n_classes])
    if n_terms:
        np.testing.assert_array_equal(g["term_count"][:n_terms], st["term_count"][:n_terms])


def _fuzz(seed, n_nodes, n_pods, extended=False):
    # k_spread keeps cpu / memory / ephemeral-storage only: extended resources send a batch to
    # k_schedule (kss_plan_podset), so the k_spread runs leave them out
    nodes, bound, pods = progfuzz.make(seed, n_nodes, n_pods, extended=extended)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    return cc, cp


@pytest.mark.parametrize("mode", ["auto", "single", "multi"])
@pytest.mark.parametrize("seed,n_nodes,n_pods", [(1, 60, 200), (2, 300, 300), (3, 700, 250), (4, 5, 40),
                                                 (5, 1000, 200)])
def test_program_fuzz_matches_oracle(seed, n_nodes, n_pods, mode):
    prof = abi.default_profile()
    cc, cp = _fuzz(seed, n_nodes, n_pods)
    ncl, nt = len(cc.classes), len(cc.terms)
    chosen_o, res, st = _oracle(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, ncl, nt)
    ctx = native.Context(prof)
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n, flags=MODES[mode])
    # one workgroup holding hundreds of nodes' rows, counts and commit table exceeds the LDS
    # budget: k_schedule takes the batch (parity is checked either way)
    assert ctx.last_kernel() == "k_spread" or (mode == "single" and n_nodes > 100)
    geo = ctx.last_geometry()
    if mode == "single":
        assert geo["shards"] == 1
    if mode == "multi" and n_nodes >= 4:
        assert geo["shards"] > 1
    _check(ctx, res, st, chosen, chosen_o, cp.n, cc.n_nodes, ncl, nt)
    ctx.close()


def test_program_fuzz_many_seeds_forced_shards(monkeypatch):
    """Twelve more seeds at 9 shards (ragged last shard)."""
    native.set_option("shards", "9")
    prof = abi.default_profile()
    for seed in range(20, 32):
        cc, cp = _fuzz(seed, 211, 150)
        ncl, nt = len(cc.classes), len(cc.terms)
        chosen_o, res, st = _oracle(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, ncl, nt)
        ctx = native.Context(prof)
        ctx.load(cc.as_struct())
        chosen = ctx.schedule_batch(cp.as_struct(), cp.n)
        assert ctx.last_kernel() == "k_spread" and ctx.last_geometry()["shards"] == 9
        _check(ctx, res, st, chosen, chosen_o, cp.n, cc.n_nodes, ncl, nt)
        ctx.close()


@pytest.mark.parametrize("fold", [True, False])
@pytest.mark.parametrize("shards", [2, 9, 40])
def test_statistics_fold_matches_oracle(fold, shards, monkeypatch):
    """Pod k+1's statistics exchange folded into pod k's argmax (spread_argmax_fold) and, with
    without KSS_FOLD (the default), the separate exchange: the fuzz mixes pods that fold (histogram-valued
    DoNotSchedule groups, inter-pod histograms and flags) with pods that cannot (node-valued
    DoNotSchedule groups) and unschedulable pods that run no argmax, so both paths alternate."""
    native.set_option("shards", str(shards))
    if fold:
        native.set_option("fold", "1")
    prof = abi.default_profile()
    on_spread = 0
    for seed in (20, 21, 22, 51):
        cc, cp = _fuzz(seed, 211, 150)
        ncl, nt = len(cc.classes), len(cc.terms)
        chosen_o, res, st = _oracle(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, ncl, nt)
        ctx = native.Context(prof)
        ctx.load(cc.as_struct())
        chosen = ctx.schedule_batch(cp.as_struct(), cp.n)
        # a program over k_spread's per-shard tables sends the batch to k_schedule (parity either way)
        on_spread += ctx.last_kernel() == "k_spread" and ctx.last_geometry()["shards"] == shards
        _check(ctx, res, st, chosen, chosen_o, cp.n, cc.n_nodes, ncl, nt)
        ctx.close()
    assert on_spread >= 3
    native.set_option("shards", 0)  # the automatic geometry (3,000 nodes do not fit 2 shards' LDS)
    s = native.Synth(3, 7, 3000, 250)  # the C3 recipe: zone DoNotSchedule, inter-pod entries
    chosen_o, res, st = _oracle(prof, s.cluster, s.pods, 250, 3000, s.cluster.n_classes, s.cluster.n_terms)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(250)
    assert ctx.last_kernel() == "k_spread"
    _check(ctx, res, st, chosen, chosen_o, 250, 3000, s.cluster.n_classes, s.cluster.n_terms)
    ctx.close()


def test_k_spread_static_chunks(monkeypatch):
    """KSS_STATIC_BYTES forces one k_static + one k_spread launch per 23 pods: the commits of
    every launch reach HBM (node rows and count rows) before the next one reads them."""
    s = native.Synth(3, 0, 2000, 300)
    native.set_option("static_bytes", str(4 * 2000 * 23))
    prof = abi.default_profile()
    chosen_o, res, st = _oracle(prof, s.cluster, s.pods, 300, 2000, s.cluster.n_classes, s.cluster.n_terms)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(300)
    assert ctx.last_kernel() == "k_spread"
    assert ctx.last_timing()[1] == 2 * ((300 + 22) // 23)
    _check(ctx, res, st, chosen, chosen_o, 300, 2000, s.cluster.n_classes, s.cluster.n_terms)
    ctx.close()


def test_k_spread_custom_profile():
    """A non-default profile (k_spread<false>: profile staged in LDS): MostAllocated,
    three BalancedAllocation resources, other plugin weights."""
    prof = abi.default_profile()
    prof.fit_strategy = abi.KSS_FIT_MOST_ALLOCATED
    prof.fit_weight[0], prof.fit_weight[1] = 3, 2
    prof.ba_n = 3
    prof.ba_res[2] = abi.KSS_RES_EPHEMERAL
    prof.weight[abi.KSS_S_POD_TOPOLOGY_SPREAD] = 5
    prof.weight[abi.KSS_S_INTER_POD_AFFINITY] = 7
    prof.weight[abi.KSS_S_TAINT_TOLERATION] = 1
    cc, cp = _fuzz(7, 400, 250)
    ncl, nt = len(cc.classes), len(cc.terms)
    chosen_o, res, st = _oracle(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, ncl, nt)
    ctx = native.Context(prof)
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n)
    assert ctx.last_kernel() == "k_spread"
    _check(ctx, res, st, chosen, chosen_o, cp.n, cc.n_nodes, ncl, nt)
    ctx.close()


def test_k_spread_and_k_schedule_agree(monkeypatch):
    s = native.Synth(3, 5, 3000, 800)
    prof = abi.default_profile()
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    a = ctx.run_staged(800).copy()
    assert ctx.last_kernel() == "k_spread"
    st_a = ctx.node_state()
    ctx.reset()
    b = ctx.schedule_batch(s.pods, 800, flags=abi.KSS_SCHED_GENERAL_KERNEL)
    assert ctx.last_kernel() == "k_schedule"
    np.testing.assert_array_equal(a, b)
    st_b = ctx.node_state()
    for k in st_a:
        np.testing.assert_array_equal(st_a[k], st_b[k])
    ctx.close()


def test_device_go_log_matches_host_port():
    """go_log_dev (k_spread's topologyNormalizingWeight) == the host port (which builds
    k_schedule's table and is pinned against the oracle) for every size up to 10^6 + 2."""
    from kss.native import lib
    import ctypes as C
    L = lib()
    L.kss_go_log_c.restype = C.c_double
    L.kss_go_log_c.argtypes = [C.c_double]
    x = np.arange(2, 1_000_003, dtype=np.float64)
    y = native.device_go_log(x)
    for k in list(range(0, 5000)) + list(range(5000, len(x), 997)):
        assert y[k] == L.kss_go_log_c(x[k]), (x[k], y[k])
    host = np.array([L.kss_go_log_c(v) for v in x[::101]])
    np.testing.assert_array_equal(y[::101], host)


def test_same_key_fixture_both_kernels():
    """The hand-derived v1.26 same-topology-key case (test_spread_same_key.py) on k_spread and,
    with every per-node record, on k_schedule."""
    import test_spread_same_key as sk
    cc, cp, _ = compile_cluster(*sk.fixture())
    prof = abi.default_profile()
    ncl, nt = len(cc.classes), len(cc.terms)
    chosen_o, res, st = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record=True,
                                          threads=8, n_classes=ncl, n_terms=nt)
    ctx = native.Context(prof, max_pods_record=cp.n)
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n)
    assert ctx.last_kernel() == "k_spread"
    _check(ctx, res, st, chosen, chosen_o, cp.n, cc.n_nodes, ncl, nt)
    ctx.reset()
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n, record=True)
    assert ctx.last_kernel() == "k_schedule"
    np.testing.assert_array_equal(chosen, chosen_o)
    for j in range(cp.n):
        r = ctx.fetch_record(j)
        np.testing.assert_array_equal(r.fail_plugin[:cc.n_nodes], res.fail_plugin[j, :cc.n_nodes])
        feas = res.fail_plugin[j, :cc.n_nodes] == 0
        if res.meta(j)["scored"]:
            np.testing.assert_array_equal(r.raw[:, :cc.n_nodes][:, feas], res.raw[j][:, :cc.n_nodes][:, feas])
    ctx.close()


@pytest.mark.parametrize("seed", [41, 42])
def test_program_fuzz_records_on_k_schedule(seed):
    """k_schedule with every per-node record on fuzzed programs (including same-key groups)."""
    prof = abi.default_profile()
    cc, cp = _fuzz(seed, 150, 120, extended=True)
    ncl, nt = len(cc.classes), len(cc.terms)
    chosen_o, res, st = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record=True,
                                          threads=8, n_classes=ncl, n_terms=nt)
    ctx = native.Context(prof, max_pods_record=cp.n)
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n, record=True, flags=abi.KSS_SCHED_FORCE_MULTI_WG)
    np.testing.assert_array_equal(chosen, chosen_o)
    for j in range(cp.n):
        r = ctx.fetch_record(j)
        m = res.meta(j)
        assert (r.chosen, r.n_feasible, r.status) == (m["chosen"], m["n_feasible"], m["status"]), j
        np.testing.assert_array_equal(r.fail_plugin[:cc.n_nodes], res.fail_plugin[j, :cc.n_nodes], err_msg=f"pod {j}")
        if m["scored"]:
            feas = res.fail_plugin[j, :cc.n_nodes] == 0
            np.testing.assert_array_equal(r.raw[:, :cc.n_nodes][:, feas], res.raw[j][:, :cc.n_nodes][:, feas],
                                          err_msg=f"pod {j}")
            np.testing.assert_array_equal(r.total[:cc.n_nodes][feas], res.total[j, :cc.n_nodes][feas])
    ctx.close()


@pytest.mark.parametrize("two_level", [1, 0, 2])
@pytest.mark.parametrize("shards", [65, 130])
def test_two_level_argmax_many_shards(two_level, shards):
    """k_spread's exchanges at more than 64 shards: the selectHost key in two levels (XCD-local
    plain stores to the XCD's rank-0 shard, then one line per XCD; tl_argmax; the default), the
    flat sweep (option spread_two_level 0), and the statistics / filter exchanges in two levels
    too (2, spread_exchange_tl), on fuzzed programs with ragged shards and over three chunk
    launches, against the C oracle."""
    native.set_option("shards", str(shards))
    native.set_option("spread_two_level", str(two_level))
    prof = abi.default_profile()
    on_spread = 0
    for seed in (20, 21, 51):
        cc, cp = _fuzz(seed, 1000, 150)
        ncl, nt = len(cc.classes), len(cc.terms)
        chosen_o, res, st = _oracle(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, ncl, nt)
        ctx = native.Context(prof)
        ctx.load(cc.as_struct())
        chosen = ctx.schedule_batch(cp.as_struct(), cp.n)
        on_spread += ctx.last_kernel() == "k_spread" and ctx.last_geometry()["shards"] == shards
        _check(ctx, res, st, chosen, chosen_o, cp.n, cc.n_nodes, ncl, nt)
        ctx.close()
    assert on_spread >= 2
    s = native.Synth(4, 3, 20000, 300)  # C4's recipe, three k_static chunks
    native.set_option("static_bytes", str(4 * 20000 * 100))
    chosen_o, res, st = _oracle(prof, s.cluster, s.pods, 300, 20000, s.cluster.n_classes, s.cluster.n_terms)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    chosen = ctx.run_staged(300)
    assert ctx.last_kernel() == "k_spread" and ctx.last_geometry()["shards"] == shards
    assert ctx.last_timing()[1] == 6
    _check(ctx, res, st, chosen, chosen_o, 300, 20000, s.cluster.n_classes, s.cluster.n_terms)
    ctx.close()
