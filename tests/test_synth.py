"""The C++ generator (csrc/kss_synth.cpp, SoA) and the Python generator (kss/synth.py,
objects -> host compiler) describe the same cluster: the C oracle schedules both identically."""
import numpy as np
import pytest

import oracle_c
from kss import abi, native, synth
from kss.compile import compile_cluster


@pytest.mark.parametrize("config,n_nodes,n_pods", [(1, 100, 400), (2, 300, 600), (3, 120, 300), (4, 150, 300),
                                                   (5, 80, 200)])
def test_cpp_and_python_generators_agree(config, n_nodes, n_pods):
    prof = abi.default_profile()
    nodes, bound, pods = synth.make_cluster(config, n_nodes, n_pods)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    ch_py, res_py, st_py = oracle_c.schedule(prof, cc.as_struct(), cp.as_struct(), cp.n, cc.n_nodes, record=True,
                                             n_classes=len(cc.classes), n_terms=len(cc.terms))
    s = native.Synth(config, 0, n_nodes, n_pods)
    ch_c, res_c, st_c = oracle_c.schedule(prof, s.cluster, s.pods, s.n_pods, s.n_nodes, record=True,
                                          n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    np.testing.assert_array_equal(ch_py, ch_c)
    np.testing.assert_array_equal(res_py.fail_plugin, res_c.fail_plugin)
    np.testing.assert_array_equal(res_py.fail_detail, res_c.fail_detail)
    np.testing.assert_array_equal(res_py.total, res_c.total)
    np.testing.assert_array_equal(st_py["requested"], st_c["requested"])
    np.testing.assert_array_equal(st_py["pod_count"], st_c["pod_count"])


def test_seed_convention():
    r = synth.SplitMix64(synth.SEED_BASE + 2)
    first = [r.next() for _ in range(3)]
    r2 = synth.SplitMix64(0x5EED0002)
    assert first == [r2.next() for _ in range(3)]
