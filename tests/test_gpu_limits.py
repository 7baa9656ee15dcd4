"""Inputs outside the device path's envelope are refused with an error, never scheduled
wrongly: malformed programs anywhere in a staged podset, profiles whose weights overflow
the packed selectHost key, and pods whose inter-pod-affinity histograms exceed the
per-pod LDS bins (status 4), on the batch path and the scenario sweep alike."""
import numpy as np
import pytest

from kss import abi, native
from kss.compile import compile_cluster

pytestmark = pytest.mark.gpu


def test_malformed_pod_beyond_n_is_rejected():
    """kss_schedule_batch stages every pod, so a bad program past n must fail the call."""
    s = native.Synth(1, 0, 50, 10)
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    import ctypes as C
    raw = C.string_at(s.pods.pods, C.sizeof(abi.Pod) * 10)
    pods_c = np.frombuffer(raw, dtype=abi.POD_DTYPE).copy()
    pods_c[9]["sel_off"] = 10 ** 6  # pod 9 refers outside the requirement pool
    bad = abi.PodSet.from_buffer_copy(bytes(s.pods))
    bad.pods = pods_c.ctypes.data_as(abi.P(abi.Pod))
    with pytest.raises(native.KssError):
        ctx.schedule_batch(bad, 5)
    ctx.close()


@pytest.mark.parametrize("weight", [21474837, 10 ** 9])
def test_profile_weight_overflow_is_refused(weight):
    prof = abi.default_profile()
    prof.weight[abi.KSS_S_TAINT_TOLERATION] = weight
    with pytest.raises(native.KssError):
        native.Context(prof)
    s = native.Synth(1, 0, 20, 5)
    with pytest.raises(native.KssError):
        native.schedule_scenarios(prof, [s.cluster], [s.pods])


def test_largest_accepted_weights_rank_correctly():
    """Σ w·100 just below 2^31: accepted, and the schedule equals the oracle's."""
    import oracle_c
    prof = abi.default_profile()
    rest = sum(prof.weight[i] for i in range(abi.KSS_NSCORE)) - prof.weight[abi.KSS_S_NODE_AFFINITY]
    prof.weight[abi.KSS_S_NODE_AFFINITY] = (2 ** 31 - 1) // 100 - rest
    s = native.Synth(2, 0, 700, 200)
    ch_o, _, st = oracle_c.schedule(prof, s.cluster, s.pods, 200, 700, record=False, threads=8)
    ctx = native.Context(prof)
    ctx.load(s.cluster)
    np.testing.assert_array_equal(ctx.schedule_batch(s.pods, 200), ch_o)
    ctx.close()


def _wide_ipa_cluster():
    """2,000 nodes with two 1,000-value (non-unique) topology keys and a pod with a
    required anti-affinity term on each: 2 x 4 x 1,001 histogram bins > LDS_BINS."""
    nodes = []
    for i in range(2000):
        nodes.append({"metadata": {"name": "n%05d" % i, "labels": {"rack": "r%d" % (i // 2), "row": "w%d" % (i % 1000)}},
                      "status": {"allocatable": {"cpu": "8", "memory": "32Gi", "pods": "110"}}})
    sel = {"matchLabels": {"app": "a"}}
    pod = {"metadata": {"name": "p", "namespace": "default", "labels": {"app": "a"}},
           "spec": {"containers": [{"name": "c", "resources": {"requests": {"cpu": "100m"}}}],
                    "affinity": {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                        {"labelSelector": sel, "topologyKey": "rack"},
                        {"labelSelector": sel, "topologyKey": "row"}]}}}}
    cc, cp, _ = compile_cluster(nodes, (), [pod])
    return cc, cp


def test_pod_over_lds_bins_is_unsupported_on_batch_and_sweep():
    cc, cp = _wide_ipa_cluster()
    ctx = native.Context(abi.default_profile())
    ctx.load(cc.as_struct())
    with pytest.raises(native.KssError) as e:
        ctx.schedule_batch(cp.as_struct(), 1)
    assert e.value.rc == -95
    ctx.close()
    with pytest.raises(native.KssError) as e:
        native.schedule_scenarios(abi.default_profile(), [cc.as_struct()], [cp.as_struct()])
    assert e.value.rc == -95
