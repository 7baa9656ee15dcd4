"""The volume plugins on the device (k_schedule; k_simple / k_spread refuse volume programs):
the hand-derived fixtures of tests/volume_fixtures.py as recorded batches, unrecorded
batches and through the per-pod eval / commit API, byte for byte against the object-level
oracle's annotations; the random volume clusters of tests/volume_fuzz.py bit-exactly against
the C oracle (every verdict, detail, score, choice, and the final vol_count / vol_attached
state); rollback and the volume delta sync; the refusals (node axis, sweeps, PostFilter)."""
import numpy as np
import pytest

import edge_fixtures as ef
import k8s_oracle
import k8s_volumes
import oracle_c
import volume_fixtures as vf
import volume_fuzz
from kss import abi, native
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu


def _want(nodes, bound, pods, st):
    o = k8s_oracle.Oracle(nodes, bound, storage=k8s_volumes.Storage(st["pvs"], st["pvcs"], st["storage_classes"],
                                                                      st["csinodes"]))
    return [o.annotations(o.schedule_one(p)) for p in pods]


def _ctx(cc, cp, n_record):
    ctx = native.Context(abi.default_profile(), max_pods_record=n_record)
    ctx.load(cc.as_struct(), names=native.make_names(cc.node_names, cc.taints, cc.scalars, cp.messages))
    return ctx


@pytest.mark.parametrize("name", sorted(vf.FIXTURES))
def test_recorded_batch_matches_hand_derived(name):
    nodes, bound, pods, expect, st = vf.FIXTURES[name]()
    want = _want(nodes, bound, pods, st)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    ps = cp.as_struct()
    ctx = _ctx(cc, cp, cp.n)
    chosen = ctx.schedule_batch(ps, cp.n, record=True)
    assert ctx.last_kernel() == "k_schedule"
    for j, exp in enumerate(expect):
        ann = ctx.format_annotations(ctx.fetch_record(j), ps, j)
        assert ann == want[j], (name, j)
        ef.check_expect(ann, exp, where=(name, j))
        sel = want[j]["scheduler-simulator/selected-node"]
        assert (cc.node_names[chosen[j]] if chosen[j] >= 0 else "") == sel, (name, j)
    ctx.close()


@pytest.mark.parametrize("name", sorted(vf.FIXTURES))
def test_unrecorded_and_per_pod_paths(name):
    nodes, bound, pods, expect, st = vf.FIXTURES[name]()
    want = _want(nodes, bound, pods, st)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    ps = cp.as_struct()
    ctx = _ctx(cc, cp, 1)
    chosen = ctx.schedule_batch(ps, cp.n)
    assert [cc.node_names[c] if c >= 0 else "" for c in chosen] == [a["scheduler-simulator/selected-node"]
                                                                    for a in want]
    ctx.reset()
    for j, exp in enumerate(expect):  # PreFilter -> kss_eval_pod, Reserve -> kss_commit
        r = ctx.eval_pod(ps, j)
        assert ctx.format_annotations(r, ps, j) == want[j], (name, j)
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
    ctx.close()


def _oracle(cc, cp, record=True):
    return oracle_c.schedule(abi.default_profile(), cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record=record,
                             n_classes=len(cc.classes), n_terms=len(cc.terms))


@pytest.mark.parametrize("seed", range(8))
def test_random_volume_clusters_match_oracle(seed):
    nodes, bound, pods, st = volume_fuzz.make(seed)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    ch_o, res, fin = _oracle(cc, cp)
    ctx = native.Context(abi.default_profile(), max_pods_record=cp.n)
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n, record=True)
    np.testing.assert_array_equal(chosen, ch_o)
    N = cc.n_nodes
    for j in range(cp.n):
        r = ctx.fetch_record(j)
        np.testing.assert_array_equal(r.fail_plugin[:N], res.fail_plugin[j], err_msg=f"pod {j}")
        np.testing.assert_array_equal(r.fail_detail[:N], res.fail_detail[j], err_msg=f"pod {j}")
        if r.scored:
            feas = res.fail_plugin[j] == 0
            np.testing.assert_array_equal(r.total[feas], res.total[j][feas], err_msg=f"pod {j}")
    vc, va = ctx.volume_state()
    np.testing.assert_array_equal(vc, fin["vol_count"])
    np.testing.assert_array_equal(va, fin["vol_attached"])
    ctx.close()


@pytest.mark.parametrize("seed,n_nodes,n_pods,flags", [(21, 400, 300, 0), (22, 3000, 200, 0),
                                                       (23, 200, 150, abi.KSS_SCHED_FORCE_SINGLE_WG)])
def test_larger_unrecorded_batches(seed, n_nodes, n_pods, flags):
    nodes, bound, pods, st = volume_fuzz.make(seed, n_nodes=n_nodes, n_bound=n_nodes, n_pods=n_pods)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    ch_o, _, fin = _oracle(cc, cp, record="meta")
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    np.testing.assert_array_equal(ctx.schedule_batch(cp.as_struct(), cp.n, flags=flags), ch_o)
    vc, va = ctx.volume_state()
    np.testing.assert_array_equal(vc, fin["vol_count"])
    np.testing.assert_array_equal(va, fin["vol_attached"])
    ctx.close()


def test_rollback_and_volume_delta():
    """kss_rollback undoes a commit's volume rows and attach counts (ForgetPod); the delta sync
    overwrites cells and a reset restores the snapshot."""
    nodes, bound, pods, st = volume_fuzz.make(3)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    ps = cp.as_struct()
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    vc0, va0 = ctx.volume_state()
    done = []
    for j in range(cp.n):
        r = ctx.eval_pod(ps, j)
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
            done.append((j, r.chosen))
    vc1, va1 = ctx.volume_state()
    assert (vc1 != vc0).any() and (va1 != va0).any()
    for j, n in reversed(done):
        ctx.rollback(ps, j, n)
    vc2, va2 = ctx.volume_state()
    np.testing.assert_array_equal(vc2, vc0)
    np.testing.assert_array_equal(va2, va0)
    R = len(cc.vol_rows)
    ctx.apply_volume_delta([0, 1], [0, R], [7, 9], overwrite=True)
    vc3, va3 = ctx.volume_state()
    assert vc3[0, 0] == 7 and va3[0, 1] == 9
    ctx.reset()
    vc4, va4 = ctx.volume_state()
    np.testing.assert_array_equal(vc4, vc0)
    np.testing.assert_array_equal(va4, va0)
    ctx.close()


def test_refusals():
    nodes, bound, pods, st = volume_fuzz.make(4)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    ps = cp.as_struct()
    with pytest.raises(native.KssError, match="volumes"):
        native.Sweep(abi.default_profile(), [cc.as_struct()], [ps])
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    j = next(i for i in range(cp.n) if cp.pods[i]["vol_len"] > 0)
    with pytest.raises(native.KssError, match="volumes"):
        ctx.postfilter_pod(ps, j)
    ctx.close()


def _binding_equal(ctx, fin):
    po, cn = ctx.binding_state()
    np.testing.assert_array_equal(po, fin["pv_owner"])
    np.testing.assert_array_equal(cn, fin["claim_node"])


@pytest.mark.parametrize("seed,n_nodes,flags", [(100, 12, 0), (103, 12, 0), (105, 12, abi.KSS_SCHED_FORCE_MULTI_WG),
                                                (108, 12, 0), (111, 12, 0), (114, 300, 0)])
def test_random_wffc_clusters_match_oracle(seed, n_nodes, flags):
    """Unbound WaitForFirstConsumer claims (binder.go FindPodVolumes / AssumePodVolumes) on random
    clusters against the C oracle: every verdict and detail (bind conflicts, the joined node + bind
    reason), choice and total, the vol_count / vol_attached state and the assume cache the batch
    leaves (pv_owner, claim_node) -- on one shard and on several (every shard applies the assume)."""
    nodes, bound, pods, st = volume_fuzz.make(seed, n_nodes=n_nodes, n_bound=max(16, n_nodes), wffc=True)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    assert cc.wclaims
    ch_o, res, fin = _oracle(cc, cp)
    ctx = native.Context(abi.default_profile(), max_pods_record=cp.n)
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n, record=True, flags=flags)
    if flags:
        assert ctx.last_geometry()["shards"] > 1
    np.testing.assert_array_equal(chosen, ch_o)
    N = cc.n_nodes
    for j in range(cp.n):
        r = ctx.fetch_record(j)
        np.testing.assert_array_equal(r.fail_plugin[:N], res.fail_plugin[j], err_msg=f"pod {j}")
        np.testing.assert_array_equal(r.fail_detail[:N], res.fail_detail[j], err_msg=f"pod {j}")
        if r.scored:
            feas = res.fail_plugin[j] == 0
            np.testing.assert_array_equal(r.total[feas], res.total[j][feas], err_msg=f"pod {j}")
    vc, va = ctx.volume_state()
    np.testing.assert_array_equal(vc, fin["vol_count"])
    np.testing.assert_array_equal(va, fin["vol_attached"])
    _binding_equal(ctx, fin)
    ctx.reset()  # the snapshot's assume cache back
    po, cn = ctx.binding_state()
    np.testing.assert_array_equal(po, cc.arrays["pv_owner"][:len(cc.pvs)])
    np.testing.assert_array_equal(cn, cc.arrays["claim_node"][:len(cc.wclaims)])
    ctx.close()


def test_wffc_per_pod_commit_rollback_and_service():
    """The drop-in's per-pod shape with WaitForFirstConsumer claims: kss_eval_pod + kss_commit
    (Reserve's AssumePodVolumes through k_wffc_commit) pod after pod equals the batch oracle and
    its assume cache; kss_rollback in reverse (RevertAssumedPodVolumes) restores the snapshot's;
    the resident service grid (eval + queued commits, every shard applying the assume) does the same."""
    nodes, bound, pods, st = volume_fuzz.make(100, wffc=True)
    cc, cp, _ = compile_cluster(nodes, bound, pods, storage=st)
    ps = cp.as_struct()
    ch_o, _, fin = _oracle(cc, cp, record="meta")
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    done = []
    for j in range(cp.n):
        r = ctx.eval_pod(ps, j)
        assert r.chosen == ch_o[j], j
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
            done.append((j, r.chosen))
    _binding_equal(ctx, fin)
    for j, n in reversed(done):
        ctx.rollback(ps, j, n)
    po, cn = ctx.binding_state()
    np.testing.assert_array_equal(po, cc.arrays["pv_owner"][:len(cc.pvs)])
    np.testing.assert_array_equal(cn, cc.arrays["claim_node"][:len(cc.wclaims)])
    ctx.reset()
    ctx.stage(ps)
    for j in range(cp.n):
        v = ctx.service_eval(j)
        assert v.chosen == ch_o[j], j
        if v.chosen >= 0:
            ctx.service_commit(j, v.chosen)
    ctx.service_stop()
    _binding_equal(ctx, fin)
    ctx.close()
