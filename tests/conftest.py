import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kube-scheduler-simulator_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def pytest_collection_modifyitems(session, config, items):
    """GPU runs: bring up torch's HIP runtime before any test loads libkss.so.  torch bundles
    its own ROCm runtime; once libkss.so's /opt/rocm runtime has opened the device first,
    torch reports "No HIP GPUs are available" (tools/torchprobe.py shows both orders), and
    the node-axis path (kss/nodeaxis.py) needs torch's device tensors."""
    if not any(it.get_closest_marker("gpu") for it in items):
        return
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.zeros(1, device="cuda")
