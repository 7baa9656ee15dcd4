import os
import sys

import pytest

# No GPU_MAX_HW_QUEUES here: the box's default (4) holds for the whole session.  The split
# grid's parts and the service grid each get a hardware queue of their own from the library
# (kss_split_config / the service's CU-masked stream), whatever the runtime's queue count.

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


CLEAN_HANDOFF = {"reloads": 0, "shadow": 0, "final": 0}


@pytest.fixture(autouse=True)
def _kss_options_reset(request):
    """Every -m gpu test starts and ends with the library's default options (kss_set_option)."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from kss import native
    native.reset_options()
    yield
    native.reset_options()


@pytest.fixture(autouse=True)
def _k_spread_handoff_clean(request, monkeypatch):
    """Every -m gpu test: after each k_spread run (run_staged / schedule_batch, split parts
    included) the node-state hand-off counters must be zero -- no prologue reload, no load the
    shadow copy answered, no last write-back that failed the final check.  A repaired hand-off
    fails the test even when the repaired results match the oracle."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    from kss import native

    def checked(fn):
        def run(self, *a, **k):
            out = fn(self, *a, **k)
            if self.last_kernel() == "k_spread":
                st = self.last_handoff_status()
                assert st == CLEAN_HANDOFF, f"k_spread hand-off not clean: {st} (diag {self.last_handoff_diag()})"
            return out
        return run

    monkeypatch.setattr(native.Context, "run_staged", checked(native.Context.run_staged))
    monkeypatch.setattr(native.Context, "schedule_batch", checked(native.Context.schedule_batch))
    yield
