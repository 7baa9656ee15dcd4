"""The SoA-level C oracle agrees with the object-level Python oracle on seeded synthetic clusters."""
import pytest

from crosscheck import run_both
from kss import synth


@pytest.mark.parametrize("config,n_nodes,n_pods", [(1, 100, 300), (1, 12, 200), (5, 40, 120)])
def test_default_profile(config, n_nodes, n_pods):
    nodes, bound, pods = synth.make_cluster(config, n_nodes, n_pods)
    run_both(nodes, bound, pods)


@pytest.mark.parametrize("n_nodes,n_pods", [(30, 150), (90, 200)])
def test_spread_and_interpod_affinity(n_nodes, n_pods):
    nodes, bound, pods = synth.make_cluster(3, n_nodes, n_pods)
    run_both(nodes, bound, pods)


def test_zone_spread_c4_recipe():
    nodes, bound, pods = synth.make_cluster(4, 60, 150)
    run_both(nodes, bound, pods)


@pytest.mark.parametrize("seed", range(8))
def test_program_fuzz(seed):
    """Every spread / inter-pod program kind (tests/progfuzz.py), the programs k_spread's
    GPU parity tests run, with per-node verdicts and raw / normalized scores compared."""
    import progfuzz
    nodes, bound, pods = progfuzz.make(1000 + seed, 70, 110)
    run_both(nodes, bound, pods)
