"""The hand-derived filter-branch fixtures (tests/edge_fixtures.py) on the device: every
reason string, PreFilterResult, system-defaulted spreading and the nodeTree tie-break through
the C-ABI -- as a recorded batch, as an unrecorded batch (the fast loop kernels), through
the per-pod eval/commit API and through the resident service grid (its k_simple-shaped
evaluation for default-profile pods) -- against the hand-derived expectations and the
object-level oracle's annotations byte for byte."""
import pytest

import edge_fixtures as ef
import k8s_oracle
from kss import abi, native
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu

PTS = abi.KSS_S_POD_TOPOLOGY_SPREAD


def _oracle(nodes, bound, pods):
    o = k8s_oracle.Oracle(nodes, bound)
    return [o.annotations(o.schedule_one(p)) for p in pods]


def _ctx(cc, n_record):
    ctx = native.Context(abi.default_profile(), max_pods_record=n_record)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars))
    return ctx


def _check(ctx, cc, ps, j, r, exp, want, where):
    ann = ctx.format_annotations(r, ps, j)
    assert ann == want, where
    pts = {nm: (int(r.raw[PTS, i]), int(r.norm[PTS, i])) for i, nm in enumerate(cc.node_names)}
    ef.check_expect(ann, exp, pts if r.scored else None, where=where)


@pytest.mark.parametrize("name", sorted(ef.FIXTURES))
def test_recorded_batch_matches_hand_derived(name):
    nodes, bound, pods, expect = ef.FIXTURES[name]()
    want = _oracle(nodes, bound, pods)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ps = cp.as_struct()
    ctx = _ctx(cc, cp.n)
    chosen = ctx.schedule_batch(ps, cp.n, record=True)
    for j, exp in enumerate(expect):
        _check(ctx, cc, ps, j, ctx.fetch_record(j), exp, want[j], (name, j))
        sel = want[j]["scheduler-simulator/selected-node"]
        assert (cc.node_names[chosen[j]] if chosen[j] >= 0 else "") == sel, (name, j)
    ctx.close()


@pytest.mark.parametrize("name", sorted(ef.FIXTURES))
def test_unrecorded_batch_same_choices(name):
    nodes, bound, pods, _ = ef.FIXTURES[name]()
    want = [a["scheduler-simulator/selected-node"] for a in _oracle(nodes, bound, pods)]
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ps = cp.as_struct()
    ctx = _ctx(cc, 0)
    chosen = ctx.schedule_batch(ps, cp.n)
    assert [cc.node_names[c] if c >= 0 else "" for c in chosen] == want, (name, ctx.last_kernel())
    ctx.close()


@pytest.mark.parametrize("name", sorted(ef.FIXTURES))
def test_per_pod_eval_commit_matches_hand_derived(name):
    nodes, bound, pods, expect = ef.FIXTURES[name]()
    want = _oracle(nodes, bound, pods)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ps = cp.as_struct()
    ctx = _ctx(cc, 1)
    for j, exp in enumerate(expect):
        r = ctx.eval_pod(ps, j)
        _check(ctx, cc, ps, j, r, exp, want[j], (name, j))
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
    ctx.close()


@pytest.mark.parametrize("name", sorted(ef.FIXTURES))
def test_service_eval_commit_matches_hand_derived(name):
    """The same fixtures through kss_service_eval / kss_service_commit: the record the grid leaves
    in the pinned host buffer formats to the oracle's annotations."""
    nodes, bound, pods, expect = ef.FIXTURES[name]()
    want = _oracle(nodes, bound, pods)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ps = cp.as_struct()
    ctx = _ctx(cc, 1)
    ctx.stage(ps)
    N = cc.n_nodes
    for j, exp in enumerate(expect):
        v = ctx.service_eval(j)
        r = native.PodResult(N)
        for k in ("fail_plugin", "fail_detail", "raw", "norm", "total"):
            getattr(r, k)[...] = getattr(v, k)
        r.s.chosen, r.s.n_feasible, r.s.best_total = v.chosen, v.n_feasible, v.best_total
        r.s.scored, r.s.status = v.scored, v.status
        _check(ctx, cc, ps, j, r, exp, want[j], (name, j, ctx.service_mode()))
        if v.chosen >= 0:
            ctx.service_commit(j, v.chosen)
    ctx.service_stop()
    ctx.close()
