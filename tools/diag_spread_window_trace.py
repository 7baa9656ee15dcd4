"""Diagnosis (trace build, make -C csrc exp EXP=trace EXP_FLAGS=-DKSS_SPREAD_TRACE=2): k_spread's
window words (GT_WIN) per shard for the first pods of a C3 batch at pct 0."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-scheduler-simulator_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
import oracle_c  # noqa: E402
from kss import abi, native  # noqa: E402
from kss.synth import SEED_BASE  # noqa: E402

p = abi.default_profile()
p.pct_nodes_to_score = 0
n, N = 4, 5000
s = native.Synth(3, SEED_BASE + 3, N, n)
ch_o, res, st = oracle_c.schedule(p, s.cluster, s.pods, n, N, record="meta", threads=8,
                                  n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms, cursor=0)
ctx = native.Context(p)
ctx.load(s.cluster)
ctx.stage(s.pods)
ch = ctx.run_staged(n)
W = ctx.last_geometry()["shards"]
L = native.lib()
fn = L.kss_trace_spread
fn.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_int32]
words = np.zeros(n * W * 128, np.int32)
fn(ctx.h, words.ctypes.data_as(C.POINTER(C.c_int32)), words.size, None, 0, None, 0)
words = words.reshape(n, W, 128)
for j in range(n):
    print("pod", j, "chosen", ch[j], ch_o[j], "oracle nf", res.meta(j)["n_feasible"])
    for w in range(W):
        print("  shard", w, list(words[j, w, 90:99]))
