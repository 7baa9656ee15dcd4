"""Probe: torch's bundled HIP runtime and libkss.so's /opt/rocm runtime in one process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator_amd"))
order = sys.argv[1]
if order == "torch-first":
    import torch
    print("torch avail", torch.cuda.is_available(), flush=True)
    x = torch.zeros(4, device="cuda")
    from kss import abi, native
    ctx = native.Context(abi.default_profile())
    print("kss ctx ok", flush=True)
    y = torch.ones(4, device="cuda")
    print("torch after kss ok", float((x + y).sum()), flush=True)
else:
    from kss import abi, native
    ctx = native.Context(abi.default_profile())
    print("kss ctx ok", flush=True)
    import torch
    print("torch avail", torch.cuda.is_available(), flush=True)
    x = torch.zeros(4, device="cuda")
    print("torch after kss ok", flush=True)
