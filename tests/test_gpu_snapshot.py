"""The generation delta sync on the device (kss/snapshot.py sync_deltas -> kss_apply_node_delta,
kss_apply_count_delta, kss_apply_port_delta): a context loaded with snapshot A and synced to
snapshot B (more bound pods: resources, PodTopologySpread / InterPodAffinity counts and
host ports) schedules B's pending pods exactly as the C oracle does on B, and a snapshot
read back from ResourcesForSnap JSON schedules like the objects it came from."""
import json

import numpy as np
import pytest

import oracle_c
import portimage_fuzz
from kss import abi, native, snapshot, synth
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu


def _oracle(cc, cp, prof=None):
    return oracle_c.schedule(prof or abi.default_profile(), cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record="meta",
                             n_classes=len(cc.classes), n_terms=len(cc.terms))


def _bind(pods, nodes, k):
    return [dict(p, spec=dict(p["spec"], nodeName=nodes[(7 * i) % len(nodes)]["metadata"]["name"]))
            for i, p in enumerate(pods[:k])]


@pytest.mark.parametrize("recipe", ["c3", "ports"])
def test_sync_deltas_equals_reload(recipe):
    if recipe == "c3":
        nodes, bound, pods = synth.make_cluster(3, n_nodes=300, n_pods=200)
    else:
        nodes, bound, pods = portimage_fuzz.make(31, n_nodes=40, n_bound=30, n_pods=80)
    cc_a, cp_a, _ = compile_cluster(nodes, bound, pods)
    cc_b, cp_b, _ = compile_cluster(nodes, bound + _bind(pods, nodes, 40), pods[40:])
    ctx = native.Context(abi.default_profile())
    ctx.load(cc_a.as_struct())
    sent = snapshot.sync_deltas(ctx, cc_a, cc_b)
    assert sent["rows"] > 0 and sent["count_cells"] > 0
    ps = cp_b.as_struct()
    ctx.stage(ps)
    chosen = ctx.run_staged(cp_b.n) if recipe == "c3" else ctx.schedule_batch(ps, cp_b.n)
    ch_o, _, st = _oracle(cc_b, cp_b)
    np.testing.assert_array_equal(chosen, ch_o)
    g = ctx.node_state()
    np.testing.assert_array_equal(g["requested"][:, :cc_b.n_nodes], st["requested"][:, :cc_b.n_nodes])
    if recipe == "ports":
        assert sent["port_rows"] > 0
        np.testing.assert_array_equal(ctx.port_state(), st["port_used"][:cc_b.n_nodes])
    ctx.close()


def test_snapshot_json_schedules_like_objects():
    nodes, bound, pods = synth.make_cluster(3, n_nodes=500, n_pods=300)
    snap = snapshot.read_snapshot(json.dumps(synth.to_resources_for_snap(nodes, bound, pods)))
    cc, cp, _ = compile_cluster(snap.nodes, snap.bound, snap.pending, snap.namespaces)
    # the simulator's profile: percentageOfNodesToScore reset to 0 (adaptive: 230 of 500 nodes)
    prof = snapshot.profile_from_config(snap.scheduler_config, cc.scalars)
    assert prof.pct_nodes_to_score == 0
    ctx = native.Context(prof)
    ctx.load(cc.as_struct())
    ctx.stage(cp.as_struct())
    ch = ctx.run_staged(cp.n)
    cc0, cp0, _ = compile_cluster(nodes, bound, pods)
    np.testing.assert_array_equal(ch, _oracle(cc0, cp0, prof)[0])
    ctx.close()
