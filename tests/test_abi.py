"""The C-ABI library loads, exports every entry point include/kss.h declares, and
its struct layouts match the ctypes mirror (no GPU needed: no compute calls)."""
import ctypes as C
import os
import re

import numpy as np

from kss import abi, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "kss.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kss_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = native.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    bound = {s[0] for s in native.SIGNATURES}
    assert set(names) <= bound, set(names) - bound


def test_struct_sizes_match_ctypes_mirror():
    L = native.lib()
    out = (C.c_int32 * 32)()
    k = L.kss_abi_sizes(out, 32)
    mirror = [abi.Cluster, abi.Req, abi.Term, abi.Spread, abi.Ipa, abi.Pod, abi.PodSet, abi.Profile, abi.PodResult,
              abi.Config, abi.Names, abi.Synth, abi.Boundset, abi.PreemptResult, abi.Vol, abi.PodView, abi.PodCView]
    assert k == len(mirror)
    for i, t in enumerate(mirror):
        assert out[i] == C.sizeof(t), (t.__name__, out[i], C.sizeof(t))


def test_default_profile_matches_reference_weights():
    p = abi.Profile()
    native.lib().kss_default_profile(C.byref(p))
    q = abi.default_profile()
    assert bytes(p) == bytes(q)
    # plugins_test.go:186-204: TT 3, NA 2, Fit 1, PTS 2, IPA 2, BA 1, ImageLocality 1
    assert list(p.weight) == [3, 2, 1, 1, 2, 2, 1, 1]


def test_go_log_table_port():
    L = native.lib()
    L.kss_go_log_c.restype = C.c_double
    L.kss_go_log_c.argtypes = [C.c_double]
    import oracle_c
    for k in range(2, 3000):
        assert L.kss_go_log_c(float(k)) == oracle_c.lib().kss_oracle_go_log(float(k))
