"""NodePorts and ImageLocality on the device (k_schedule; k_simple / k_spread refuse these pods,
kss_plan_podset names the reason) against the C oracle on the random clusters of
tests/portimage_fuzz.py: recorded batches (every verdict and raw / normalised score),
unrecorded batches, the per-pod eval / commit API, rollback of UsedPorts, the port delta
sync and the refusals (node axis, sweeps, PostFilter with host ports)."""
import numpy as np
import pytest

import oracle_c
import portimage_fuzz
from kss import abi, native
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu


def _compiled(seed, **kw):
    nodes, bound, pods = portimage_fuzz.make(seed, **kw)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    return cc, cp


def _oracle(cc, cp, record=True):
    return oracle_c.schedule(abi.default_profile(), cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record=record,
                             n_classes=len(cc.classes), n_terms=len(cc.terms))


@pytest.mark.parametrize("seed", range(6))
def test_recorded_batch_matches_oracle(seed):
    cc, cp = _compiled(seed)
    ch_o, res, st = _oracle(cc, cp)
    ctx = native.Context(abi.default_profile(), max_pods_record=cp.n)
    ctx.load(cc.as_struct())
    ps = cp.as_struct()
    chosen = ctx.schedule_batch(ps, cp.n, record=True)
    assert ctx.last_kernel() == "k_schedule"
    np.testing.assert_array_equal(chosen, ch_o)
    for j in range(cp.n):
        r = ctx.fetch_record(j)
        np.testing.assert_array_equal(r.fail_plugin[:cc.n_nodes], res.fail_plugin[j], err_msg=f"pod {j}")
        if r.scored:
            feas = res.fail_plugin[j] == 0
            np.testing.assert_array_equal(r.raw[:, feas], res.raw[j][:, feas], err_msg=f"pod {j}")
            np.testing.assert_array_equal(r.norm[:, feas], res.norm[j][:, feas], err_msg=f"pod {j}")
            np.testing.assert_array_equal(r.total[feas], res.total[j][feas], err_msg=f"pod {j}")
    np.testing.assert_array_equal(ctx.port_state(), st["port_used"][:cc.n_nodes])
    np.testing.assert_array_equal(ctx.node_state()["requested"][:, :cc.n_nodes], st["requested"][:, :cc.n_nodes])
    ctx.close()


@pytest.mark.parametrize("seed,n_nodes,n_pods,flags", [(11, 300, 200, 0),
                                                       (12, 2000, 300, 0),
                                                       (13, 300, 120, abi.KSS_SCHED_FORCE_SINGLE_WG)])
def test_unrecorded_batch_matches_oracle(seed, n_nodes, n_pods, flags):
    cc, cp = _compiled(seed, n_nodes=n_nodes, n_bound=n_nodes, n_pods=n_pods)
    ch_o, _, st = _oracle(cc, cp, record="meta")
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    chosen = ctx.schedule_batch(cp.as_struct(), cp.n, flags=flags)
    np.testing.assert_array_equal(chosen, ch_o)
    np.testing.assert_array_equal(ctx.port_state(), st["port_used"][:cc.n_nodes])
    ctx.close()


def test_per_pod_api_commit_rollback_and_delta():
    cc, cp = _compiled(21)
    ch_o, res, st = _oracle(cc, cp)
    ps = cp.as_struct()
    ctx = native.Context(abi.default_profile(), max_pods_record=1)
    ctx.load(cc.as_struct())
    used0 = ctx.port_state().copy()
    for j in range(cp.n):
        r = ctx.eval_pod(ps, j)
        assert r.chosen == ch_o[j], j
        np.testing.assert_array_equal(r.fail_plugin[:cc.n_nodes], res.fail_plugin[j], err_msg=f"pod {j}")
        if r.chosen >= 0:
            ctx.commit(ps, j, r.chosen)
    np.testing.assert_array_equal(ctx.port_state(), st["port_used"][:cc.n_nodes])
    # Unreserve in reverse order restores the snapshot's UsedPorts (HostPortInfo.Remove)
    for j in reversed(range(cp.n)):
        if ch_o[j] >= 0:
            ctx.rollback(ps, j, int(ch_o[j]))
    np.testing.assert_array_equal(ctx.port_state(), used0)
    # an externally bound pod's ports (kss_apply_port_delta), then reset restores the snapshot
    ctx.apply_port_delta([0, 1], [1, 3])
    got = ctx.port_state()
    assert got[0] == 1 and got[1] == 3
    ctx.reset()
    np.testing.assert_array_equal(ctx.port_state(), used0)
    ctx.close()


def test_plan_and_refusals():
    cc, cp = _compiled(5)
    plan = native.plan_podset(cc.as_struct(), cp.as_struct())
    assert plan["kernel"] == "k_schedule" and "host ports" in plan["reason"], plan
    ps = cp.as_struct()
    with pytest.raises(native.KssError):  # the sweep packs no port / image columns
        native.Sweep(abi.default_profile(), [cc.as_struct()], [ps])
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    j = next(i for i in range(cp.n) if cp.pods[i]["port_conflict"])
    with pytest.raises(native.KssError):
        ctx.postfilter_pod(ps, j)
    ctx.close()
