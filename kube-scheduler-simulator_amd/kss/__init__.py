"""kss — MI355X-native Filter/Score evaluator for kube-scheduler-simulator's scheduling cycle.

Host-side Python package: the object -> SoA compiler (``kss.compile``), the
ctypes binding of the C ABI (``kss.native``, include/kss.h), and the
framework-interface mirror (``kss.framework``).  The compute path is the HIP
library ``libkss.so`` built from ``csrc/``; there is no CPU fallback.
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
