"""kss — MI355X-native Filter/Score evaluator for kube-scheduler-simulator's scheduling cycle.

Host-side Python package: the object -> SoA compiler (``kss.compile``), the ctypes binding
of the C ABI (``kss.native``, include/kss.h), snapshot / scheduler-config I/O
(``kss.snapshot``), and the multi-GPU drivers (``kss.split``: the node axis as one split
grid; ``kss.nodeaxis``: the per-pod RCCL variant).  The compute path is the HIP library
``libkss.so`` built from ``csrc/``; there is no CPU fallback.
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
