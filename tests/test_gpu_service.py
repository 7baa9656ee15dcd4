"""The per-pod service grid (kss_service_*: a resident grid taking commands from a pinned host
ring) against the launch-per-call per-pod API (kss_eval_pod_view / kss_commit): the same
record (verdicts, details, raw / normalised scores, totals) and choice for every pod of
default-profile, spread + inter-pod, port / image and volume workloads, commits and
rollbacks in between, the grid restarting after its idle exit, and the other entry points
stopping it first."""
import time

import numpy as np
import pytest

import volume_fuzz
from kss import abi, native
from kss.compile import compile_cluster
from kss.synth import SEED_BASE

pytestmark = pytest.mark.gpu


def _same(a, b, N, where):
    assert (a.chosen, a.n_feasible, a.scored, a.status, a.best_total) == \
           (b.chosen, b.n_feasible, b.scored, b.status, b.best_total), where
    np.testing.assert_array_equal(a.fail_plugin[:N], b.fail_plugin[:N], err_msg=str(where))
    np.testing.assert_array_equal(a.fail_detail[:N], b.fail_detail[:N], err_msg=str(where))
    if a.scored:
        feas = a.fail_plugin[:N] == 0
        np.testing.assert_array_equal(a.raw[:, :N][:, feas], b.raw[:, :N][:, feas], err_msg=str(where))
        np.testing.assert_array_equal(a.norm[:, :N][:, feas], b.norm[:, :N][:, feas], err_msg=str(where))
        np.testing.assert_array_equal(a.total[:N][feas], b.total[:N][feas], err_msg=str(where))


def _copy(v):
    import types
    out = types.SimpleNamespace()
    for k in ("fail_plugin", "fail_detail", "raw", "norm", "total"):
        setattr(out, k, None if getattr(v, k) is None else np.array(getattr(v, k)))
    for k in ("chosen", "n_feasible", "scored", "status", "best_total"):
        setattr(out, k, getattr(v, k))
    return out


def _compare(cluster, pods, n, rollback_every=0):
    """Service eval + commit vs eval_pod_view + commit, pod after pod: the launch-per-call
    sequence runs first, to completion, then the service sequence.  (Interleaving two contexts
    in one process would put the reference context's launches behind the resident grid
    whenever their streams share a hardware queue: they would wait for its idle exit.)"""
    ref = native.Context(abi.default_profile())
    ref.load(cluster)
    N = ref.n_nodes
    want = []
    for j in range(n):
        w = _copy(ref.eval_pod_view(pods, j))
        want.append(w)
        if w.chosen >= 0:
            ref.commit(pods, j, w.chosen)
            if rollback_every and j % rollback_every == 0:
                ref.rollback(pods, j, w.chosen)
    st_r = ref.node_state()
    ref.close()
    svc = native.Context(abi.default_profile())
    svc.load(cluster)
    svc.stage(pods)
    for j in range(n):
        got = svc.service_eval(j)
        _same(got, want[j], N, j)
        if j == 0:
            mode = svc.service_mode()
        if want[j].chosen >= 0:
            svc.service_commit(j, want[j].chosen)
            if rollback_every and j % rollback_every == 0:
                svc.service_rollback(j, want[j].chosen)
    svc.service_stop()
    st_s = svc.node_state()
    for k in ("requested", "nonzero", "pod_count"):
        np.testing.assert_array_equal(st_s[k], st_r[k], err_msg=k)
    svc.close()
    return mode if n else -1


@pytest.mark.parametrize("config,n_nodes,n_pods", [(2, 5000, 120), (1, 100, 200), (3, 2000, 80), (4, 6000, 60)])
def test_service_matches_per_pod_api(config, n_nodes, n_pods):
    """Default-profile configs (1, 2) run the k_simple-shaped evaluation, program configs (3, 4)
    the general chain; both equal the per-pod API record for record."""
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    mode = _compare(s.cluster, s.pods, n_pods, rollback_every=7)
    assert (mode in (1, 2)) if config in (1, 2) else mode == 0, mode
    s.close()


@pytest.mark.parametrize("config,n_nodes,n_pods", [(2, 5000, 60), (1, 100, 80)])
def test_general_service_matches_per_pod_api(config, n_nodes, n_pods, monkeypatch):
    """KSS_SERVICE_GENERAL=1 keeps default-profile pods on the general chain (the comparison
    the per-pod bench reports)."""
    native.set_option("service_general", "1")
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    assert _compare(s.cluster, s.pods, n_pods, rollback_every=5) == 0
    s.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_service_with_volumes(seed):
    nodes, bound, pods, st = volume_fuzz.make(seed, n_nodes=300, n_bound=300, n_pods=60)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    _compare(cc.as_struct(), cp.as_struct(), cp.n, rollback_every=5)


def test_service_restarts_after_idle_exit_and_yields_to_other_calls():
    s = native.Synth(2, SEED_BASE + 2, 3000, 40)
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    a = _copy(ctx.service_eval(0))
    time.sleep(2.5)  # the grid leaves after ~1 s idle
    b = ctx.service_eval(0)  # restarted transparently
    _same(b, a, 3000, "after idle exit")
    ctx.service_commit(0, a.chosen)
    st = ctx.node_state()  # stops the grid first: the commit is in the state read back
    assert st["pod_count"][a.chosen] == s.cluster.pod_count[a.chosen] + 1
    c = ctx.eval_pod_view(s.pods, 1)  # the launch-per-call path works after the service
    d = ctx.service_eval(1)  # and the service starts again on the same state
    _same(d, _copy(c), 3000, "after the per-pod API")
    ctx.close()
    s.close()


def test_commit_after_idle_exit_is_applied():
    """A commit posted after the grid left idle is not dropped: the grid is relaunched for it
    (ADVICE r3), also when the next call stops the service right away."""
    s = native.Synth(2, SEED_BASE + 2, 3000, 40)
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    a = _copy(ctx.service_eval(0))
    time.sleep(2.5)  # the grid leaves after ~1 s idle
    ctx.service_commit(0, a.chosen)
    st = ctx.node_state()  # stops the service: the queued commit must be in the state
    assert st["pod_count"][a.chosen] == s.cluster.pod_count[a.chosen] + 1
    b = _copy(ctx.service_eval(1))
    time.sleep(2.5)
    ctx.service_commit(1, b.chosen)
    time.sleep(2.5)  # the relaunched grid leaves idle again after taking the commit
    ctx.service_rollback(1, b.chosen)
    ctx.service_stop()
    st2 = ctx.node_state()
    assert st2["pod_count"][a.chosen] == s.cluster.pod_count[a.chosen] + 1
    if b.chosen != a.chosen:
        assert st2["pod_count"][b.chosen] == s.cluster.pod_count[b.chosen]
    ctx.close()
    s.close()


@pytest.mark.parametrize("config,n_nodes,n_pods", [(2, 5000, 40), (3, 2000, 30), (4, 6000, 24)])
def test_service_compact_record_equals_full(config, n_nodes, n_pods):
    """kss_service_eval_compact (scores narrowed on the device: int32 raw / total, uint8
    normalised) against kss_service_eval on the same state, pod after pod with commits in
    between; the two records are asked in both orders and with a field subset, so the
    host-segment bookkeeping of each record (rows resent only when they changed) is crossed.
    The wide fallback (a value outside the narrow types) is not reached by any in-range
    workload: check_profile bounds the totals and the raw scores stay far below 2^31."""
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    svc = native.Context(abi.default_profile())
    svc.load(s.cluster)
    svc.stage(s.pods)
    N = svc.n_nodes
    sub = abi.KSS_FIELD_FAIL | abi.KSS_FIELD_TOTAL
    for j in range(n_pods):
        fields = sub if j % 5 == 4 else abi.KSS_FIELD_ALL
        if j % 2:
            c = _copy(svc.service_eval_compact(j, fields))
            f = _copy(svc.service_eval(j, fields))
        else:
            f = _copy(svc.service_eval(j, fields))
            c = _copy(svc.service_eval_compact(j, fields))
        assert (c.chosen, c.n_feasible, c.scored, c.status, c.best_total) == \
               (f.chosen, f.n_feasible, f.scored, f.status, f.best_total), j
        for k in ("fail_plugin", "fail_detail", "raw", "norm", "total"):
            a, b = getattr(c, k), getattr(f, k)
            assert (a is None) == (b is None), (j, k)
            if a is not None:
                assert a.dtype == {"fail_plugin": np.uint8, "fail_detail": np.uint16, "raw": np.int32,
                                   "norm": np.uint8, "total": np.int32}[k], (j, k, a.dtype)
                np.testing.assert_array_equal(a[..., :N].astype(np.int64), b[..., :N].astype(np.int64),
                                              err_msg=f"pod {j} {k}")
        if f.chosen >= 0:
            svc.service_commit(j, f.chosen)
    svc.service_stop()
    svc.close()


def _oracle_records(cluster, pods, n, rollback_every, n_classes=0, n_terms=0, prof=None):
    """The C oracle's records for the service sequence: pod j evaluated on the state every earlier
    commit left; a commit the sequence rolled back is not assumed (skip_commit)."""
    import oracle_c
    skip = np.zeros(n, np.uint8)
    if rollback_every:
        skip[::rollback_every] = 1
    return oracle_c.schedule(prof or abi.default_profile(), cluster, pods, n, cluster.n_nodes, threads=8, record=True,
                             n_classes=n_classes, n_terms=n_terms, skip_commit=skip)


@pytest.mark.parametrize("config,n_nodes,n_pods,pct", [(2, 5000, 100, 100), (1, 100, 150, 100), (3, 2000, 70, 100),
                                                       (4, 6000, 50, 100), (2, 5000, 150, 0), (2, 2000, 120, 30),
                                                       (1, 180, 200, 0), (3, 2000, 60, 0)])
def test_service_records_match_c_oracle(config, n_nodes, n_pods, pct):
    """The service's full records straight against the C oracle: every pod's
    chosen node, outcome, per-node verdicts and details, raw and normalised scores and weighted
    totals over the kept nodes, with the commit / rollback sequence replayed in the oracle
    (rolled-back pods evaluated, not assumed), the cursor and the final node state -- on the
    k_simple-shaped evaluation (configs 1, 2; at pct < 100 with the window, svc_window: the
    stopping node recorded as passed and dropped, the nodes after it unevaluated) and the general
    chain (3, 4: spread and inter-pod programs)."""
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    rb = 7
    prof = abi.default_profile()
    prof.pct_nodes_to_score = pct
    ch_o, res, st = _oracle_records(s.cluster, s.pods, n_pods, rb, s.cluster.n_classes, s.cluster.n_terms, prof)
    svc = native.Context(prof)
    svc.load(s.cluster)
    svc.stage(s.pods)
    N = svc.n_nodes
    for j in range(n_pods):
        got = svc.service_eval(j)
        m = res.meta(j)
        assert (got.chosen, got.n_feasible, got.scored, got.status) == \
               (m["chosen"], m["n_feasible"], m["scored"], m["status"]), (j, m)
        np.testing.assert_array_equal(got.fail_plugin[:N], res.fail_plugin[j, :N], err_msg=f"pod {j} verdicts")
        np.testing.assert_array_equal(got.fail_detail[:N], res.fail_detail[j, :N], err_msg=f"pod {j} details")
        if j == 0:
            mode = svc.service_mode()
        if m["scored"]:
            assert got.best_total == m["best_total"], j
            feas = (res.fail_plugin[j, :N] == 0) & (res.fail_detail[j, :N] != abi.KSS_PASS_NOT_KEPT)
            np.testing.assert_array_equal(got.raw[:, :N][:, feas], res.raw[j][:, :N][:, feas], err_msg=f"pod {j} raw")
            np.testing.assert_array_equal(got.norm[:, :N][:, feas], res.norm[j][:, :N][:, feas], err_msg=f"pod {j} norm")
            np.testing.assert_array_equal(got.total[:N][feas], res.total[j, :N][feas], err_msg=f"pod {j} total")
        if got.chosen >= 0:
            svc.service_commit(j, got.chosen)
            if j % rb == 0:
                svc.service_rollback(j, got.chosen)
    svc.service_stop()
    assert svc.next_start_node_index() == st["next_start"]
    assert (mode in (1, 2)) if config in (1, 2) else mode == 0, mode
    g = svc.node_state()
    for k in ("requested", "nonzero", "pod_count"):
        np.testing.assert_array_equal(g[k][..., :N], st[k][..., :N], err_msg=k)
    if s.cluster.n_classes:
        np.testing.assert_array_equal(g["class_count"][:s.cluster.n_classes], st["class_count"][:s.cluster.n_classes])
    svc.close()
    s.close()
