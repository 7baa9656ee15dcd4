"""Diagnosis helper for the many-chunk split test (test infrastructure): when the library is
the k_spread trace build (make -C kube-scheduler-simulator_amd/csrc exp EXP=tl
EXP_FLAGS=-DKSS_SPREAD_TRACE=2, loaded with KSS_LIB=tl), report for the last run every
nonzero count a shard loaded in a chunk's prologue or wrote back in its epilogue that differs
from the counts replayed from the device's own choices, with the XCD each shard's workgroup
ran on in every chunk.  With the product library it reports nothing."""
import ctypes as C

import numpy as np

from kss import native

TW = 128
GT_XCC = 89
TLIST = 1 << 20


def available():
    return hasattr(native.lib(), "kss_trace_spread")


def fetch(ctx, n, W):
    fn = native.lib().kss_trace_spread
    P = C.POINTER
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, P(C.c_int32), C.c_int64, P(C.c_int32), C.c_int64, P(C.c_int32), C.c_int32]
    words = np.zeros(n * W * TW, np.int32)
    lst = np.zeros(4 + 4 * TLIST, np.int32)
    rows = np.full(65536, -1, np.int32)
    fn(ctx.h, words.ctypes.data_as(P(C.c_int32)), words.size, lst.ctypes.data_as(P(C.c_int32)), lst.size,
       rows.ctypes.data_as(P(C.c_int32)), rows.size)
    used = min(int(lst[0]), TLIST)
    return words.reshape(n, W, TW), lst[4:4 + 4 * used].reshape(used, 4), rows[rows >= 0]


def replay(cls, chosen, init_cc, n):
    """Class counts before each pod k, as {(row, node): count}."""
    cur = {(int(r), int(c)): int(init_cc[r, c]) for r, c in zip(*np.nonzero(init_cc))}
    out = [dict(cur)]
    for k in range(n):
        if chosen[k] >= 0:
            key = (int(cls[k]), int(chosen[k]))
            cur[key] = cur.get(key, 0) + 1
        out.append(dict(cur))
    return out


def report(sp, pods, init_cc, n, wl, per_chunk, part_rows):
    """Print the per-chunk count mismatches of every part (trace build only)."""
    if not available():
        return
    W = len(sp.ctxs) * wl
    cls = np.array([pods.pods[j].cls for j in range(n)])
    per = -(-sp.n_nodes // W)
    for p, ctx in enumerate(sp.ctxs):
        words, lst, rows = fetch(ctx, n, W)
        chosen = ctx.fetch_meta(n)[:, 0]
        exp = replay(cls, chosen, init_cc, n)
        lo, hi = part_rows(sp.n_nodes, len(sp.ctxs), wl, p)
        res = set(int(r) for r in rows)
        xcc = {}
        for k0 in range(0, n, per_chunk):
            for w in range(p * wl, (p + 1) * wl):
                xcc[(k0 // per_chunk, w)] = int(words[k0, w, GT_XCC]) - 16
        for k0 in range(0, n, per_chunk):
            k1 = min(n, k0 + per_chunk)
            for t, kk, what in ((k0, k0, "loaded"), (-1 - k1, k1, "written back")):
                got = {(int(e[1]), int(e[2])): int(e[3]) for e in lst if e[0] == t and lo <= e[2] < hi}
                want = {key: v for key, v in exp[kk].items() if v and key[0] in res and lo <= key[1] < hi}
                bad = [(key, got.get(key, 0), want.get(key, 0)) for key in sorted(set(got) | set(want))
                       if got.get(key, 0) != want.get(key, 0)]
                for key, g, wv in bad[:6]:
                    sh = key[1] // per
                    c = k0 // per_chunk
                    print(f"part {p} chunk {c} (pods {k0}..{k1 - 1}): count {what} (row {key[0]}, node {key[1]}) = {g}, "
                          f"replay {wv}; shard {sh} on XCD {[xcc.get((cc, sh)) for cc in range(max(0, c - 2), c + 2)]} "
                          f"(chunks {max(0, c - 2)}..{c + 1})")
