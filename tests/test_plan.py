"""Host-only kernel planning (kss_plan_podset): which sequential-loop kernel a batch's pod
programs admit, and the reason when k_spread is ruled out (no GPU needed)."""
import pytest

import progfuzz
from kss import abi, native
from kss.compile import compile_cluster


@pytest.mark.parametrize("config,kernel", [(1, "k_simple"), (2, "k_simple"), (3, "k_spread"), (4, "k_spread"),
                                           (5, "k_simple")])
def test_baseline_configs(config, kernel):
    s = native.Synth(config, 0, 300, 200)
    assert native.plan_podset(s.cluster, s.pods) == {"kernel": kernel, "pod": -1, "reason": "eligible"}


@pytest.mark.parametrize("seed,n_nodes,n_pods", [(1, 60, 200), (2, 300, 300), (3, 700, 250), (5, 1000, 200)])
def test_program_fuzz_batches_take_k_spread(seed, n_nodes, n_pods):
    """The batches test_gpu_spread.py runs: every one admitted by k_spread (the GPU tests
    assert the kernel that ran)."""
    nodes, bound, pods = progfuzz.make(seed, n_nodes, n_pods, extended=False)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    assert native.plan_podset(cc.as_struct(), cp.as_struct())["kernel"] == "k_spread"


def test_extended_resources_stay_on_the_loop_kernels():
    """Extended (scalar) resources: k_simple / k_spread filter and commit them in LDS."""
    nodes, bound, pods = progfuzz.make(1, 60, 200, n_extended=4)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    assert len(cc.scalars) == 4 and progfuzz.R_GPU in cc.scalars
    assert native.plan_podset(cc.as_struct(), cp.as_struct())["kernel"] == "k_spread"
    nodes, bound, pods = progfuzz.make(2, 60, 200, n_extended=2, programs=False)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    assert len(cc.scalars) == 2
    assert native.plan_podset(cc.as_struct(), cp.as_struct())["kernel"] == "k_simple"


def test_refusal_names_pod_and_reason():
    """Required anti-affinity over five topology keys exceeds the four key slots of a pod
    program: k_schedule only, with the pod and the reason named."""
    nodes, bound, pods = progfuzz.make(9, 20, 5, extended=False)
    keys = (progfuzz.K_ZONE, progfuzz.K_RACK, progfuzz.K_HOST, progfuzz.K_ITYPE, "example.com/none")
    pods[3]["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "a1"}}, "topologyKey": k} for k in keys]}}
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    plan = native.plan_podset(cc.as_struct(), cp.as_struct())
    assert plan == {"kernel": "k_schedule", "pod": 3, "reason": "more than 4 inter-pod-affinity topology keys"}


def test_profile_aware_plan():
    """kss_plan_podset_ex: percentageOfNodesToScore below 100 on 100+ nodes (the window) keeps
    k_simple for pods without a PreFilterResult list (simple_sync_win) and k_spread under the
    default profile (spread_schedule WIN), and rules out name-listed pods and k_spread under a
    custom profile; a profile that scores an extended resource the cluster has rules out both
    loop kernels; otherwise it answers as kss_plan_podset."""
    s = native.Synth(2, 0, 500, 50)
    assert native.plan_podset(s.cluster, s.pods)["kernel"] == "k_simple"
    for pct in (0, 30, 99):
        p = abi.default_profile()
        p.pct_nodes_to_score = pct
        assert native.plan_podset(s.cluster, s.pods, p)["kernel"] == "k_simple"
    small = native.Synth(2, 0, 99, 20)  # fewer than 100 nodes: no window at all
    p = abi.default_profile()
    p.pct_nodes_to_score = 0
    assert native.plan_podset(small.cluster, small.pods, p)["kernel"] == "k_simple"
    # programs keep k_spread under the default profile; a custom profile and PreFilterResult node
    # lists keep the window on k_schedule
    from kss import synth
    from test_oracle_crosscheck import with_name_sets
    nodes, bound, pods = synth.make_cluster(3, 300, 40)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    assert native.plan_podset(cc.as_struct(), cp.as_struct())["kernel"] == "k_spread"
    assert native.plan_podset(cc.as_struct(), cp.as_struct(), p)["kernel"] == "k_spread"
    pc = abi.default_profile()
    pc.pct_nodes_to_score = 0
    pc.weight[abi.KSS_S_TAINT_TOLERATION] = 5
    r = native.plan_podset(cc.as_struct(), cp.as_struct(), pc)
    assert r["kernel"] == "k_schedule" and "percentageOfNodesToScore" in r["reason"], r
    nodes, bound, pods = synth.make_cluster(2, 300, 40)
    pods = with_name_sets(pods, [n["metadata"]["name"] for n in nodes], every=5, size=120)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    assert native.plan_podset(cc.as_struct(), cp.as_struct())["kernel"] == "k_simple"
    r = native.plan_podset(cc.as_struct(), cp.as_struct(), p)
    assert r["kernel"] == "k_schedule" and "PreFilterResult" in r["reason"], r
    assert native.plan_podset(s.cluster, s.pods, abi.default_profile())["kernel"] == "k_simple"
    nodes, bound, pods = progfuzz.make(2, 60, 200, n_extended=2, programs=False)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    p = abi.default_profile()
    p.fit_n = 3
    p.fit_res[2] = abi.KSS_RES_SCALAR0
    p.fit_weight[2] = 1
    r = native.plan_podset(cc.as_struct(), cp.as_struct(), p)
    assert r["kernel"] == "k_schedule" and "extended" in r["reason"], r
    assert native.plan_podset(cc.as_struct(), cp.as_struct(), abi.default_profile())["kernel"] == "k_simple"


def test_profile_pct_range_is_checked():
    s = native.Synth(2, 0, 50, 5)
    p = abi.default_profile()
    p.pct_nodes_to_score = 101
    with pytest.raises(native.KssError, match="percentageOfNodesToScore"):
        native.plan_podset(s.cluster, s.pods, p)
