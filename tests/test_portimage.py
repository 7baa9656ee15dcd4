"""NodePorts and ImageLocality on random clusters: the object-level oracle (HostPortInfo over
objects, ImageStates built node by node) and the C oracle over the compiled dictionaries agree
on every verdict, raw / normalised score and choice (tests/portimage_fuzz.py)."""
import numpy as np
import pytest

import portimage_fuzz
from crosscheck import run_both
from kss import abi
from kss.compile import compile_cluster, ports_conflict


@pytest.mark.parametrize("seed", range(12))
def test_oracles_agree_on_ports_and_images(seed):
    nodes, bound, pods = portimage_fuzz.make(seed)
    cc, cp, chosen, res = run_both(nodes, bound, pods)
    assert cc.ports and cc.images  # the recipe reaches both plugins
    il = res.raw[:, abi.KSS_S_IMAGE_LOCALITY, :]
    assert (il > 0).any()
    assert (res.fail_plugin == abi.KSS_F_NODE_PORTS).any()


def test_port_conflict_rule():
    """HostPortInfo.CheckConflict: a wildcard want meets every IP, a specific IP only the
    wildcard or itself; protocol and port must match."""
    assert ports_conflict(("0.0.0.0", "TCP", 80), ("10.0.0.1", "TCP", 80))
    assert ports_conflict(("10.0.0.1", "TCP", 80), ("0.0.0.0", "TCP", 80))
    assert ports_conflict(("10.0.0.1", "TCP", 80), ("10.0.0.1", "TCP", 80))
    assert not ports_conflict(("10.0.0.1", "TCP", 80), ("10.0.0.2", "TCP", 80))
    assert not ports_conflict(("0.0.0.0", "UDP", 80), ("0.0.0.0", "TCP", 80))
    assert not ports_conflict(("0.0.0.0", "TCP", 81), ("0.0.0.0", "TCP", 80))


def test_compiled_masks():
    nodes, bound, pods = portimage_fuzz.make(3)
    cc, cp, _ = compile_cluster(nodes, bound, pods)
    used = cc.arrays["port_used"][:cc.n_nodes]
    assert (used >> np.uint64(len(cc.ports)) == 0).all()
    for rec in cp.pods:
        add, conf = int(rec["port_add"]), int(rec["port_conflict"])
        assert add & ~conf == 0  # a port always conflicts with itself
        if rec["img_len"]:
            rows = cp.ints[rec["img_off"]:rec["img_off"] + rec["img_len"]]
            assert ((0 <= rows) & (rows < len(cc.images))).all()
            assert rec["img_len"] <= rec["n_containers"]
