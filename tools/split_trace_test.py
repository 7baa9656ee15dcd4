"""Diagnosis of the many-chunk split-grid failure (tests/test_gpu_split.py::
test_parts_over_many_chunks[4-6000-200-24-16]) with the k_spread trace build:

    make -C kube-scheduler-simulator_amd/csrc exp EXP=trace EXP_FLAGS=-DKSS_SPREAD_TRACE=1
    KSS_LIB=trace python -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py \
        tools/split_trace_test.py -m gpu -k 'spread or split or trace' -s

(the spread modules first: the failure showed in first processes that ran them).  Every run
replays the class counts on the host from the device's own choices and checks, per part:
  * every nonzero count a shard loaded in a chunk's prologue, and every one it wrote back in
    the epilogue, against the replayed counts at that chunk's first / last pod (and that no
    expected nonzero count is missing from either list);
  * the count the winner shard held at each commit, against the replay;
  * per (pod, shard): staged record / static words / label ids against HBM, a count that
    changed between two reads around the statistics pass, local bins against run 0.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "kube-scheduler-simulator_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
import oracle_c  # noqa: E402
from kss import abi, native, split
from kss.synth import SEED_BASE

pytestmark = pytest.mark.gpu
TW = 128
GT = dict(LOCAL=0, XBINS=32, MINIMA=64, EPOCH=69, REREAD=71, BAD_ST=72, BAD_REC=73, BAD_LBL=74, KEY=75, NF=78,
          CHOSEN=79, CMT=80, PRO=88)
TLIST = 1 << 20


def _fetch(ctx, n, W):
    L = native.lib()
    if not hasattr(L, "kss_trace_spread"):
        pytest.skip("not the trace build (KSS_LIB=trace)")
    fn = L.kss_trace_spread
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


def _replay(cls, chosen, init_cc, n):
    """Class counts before each pod k (dict of (row, node) -> count), from the choices."""
    cur = {(int(r), int(c)): int(init_cc[r, c]) for r, c in zip(*np.nonzero(init_cc))}
    out = [dict(cur)]
    for k in range(n):
        if chosen[k] >= 0:
            key = (int(cls[k]), int(chosen[k]))
            cur[key] = cur.get(key, 0) + 1
        out.append(dict(cur))
    return out


def _check_list(tag, lst, exp, rows, lo, hi, chunk, n):
    """Count-list entries against the replay: loads at k0 vs exp[k0], stores at k1 vs exp[k1]."""
    out = []
    res = set(int(r) for r in rows)
    for k0 in range(0, n, chunk):
        k1 = min(n, k0 + chunk)
        for t, kk, what in ((k0, k0, "loaded"), (-1 - k1, k1, "written back")):
            got = {(int(e[1]), int(e[2])): int(e[3]) for e in lst if e[0] == t and lo <= e[2] < hi}
            want = {key: v for key, v in exp[kk].items() if v and key[0] in res and lo <= key[1] < hi}
            bad = [(key, got.get(key, 0), want.get(key, 0)) for key in sorted(set(got) | set(want))
                   if got.get(key, 0) != want.get(key, 0)]
            if bad:
                out.append(f"{tag} chunk {k0 // chunk} (pods {k0}..{k1 - 1}): counts {what} differing "
                           f"((row, node), device, replay) {bad[:8]}")
    return out


@pytest.mark.parametrize("config,n_nodes,n_pods,per_chunk,wl,runs", [(4, 6000, 200, 24, 16, 3)])
def test_trace_many_chunks(monkeypatch, config, n_nodes, n_pods, per_chunk, wl, runs):
    monkeypatch.setenv("KSS_STATIC_BYTES", str(4 * n_nodes * per_chunk))
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, res, st = oracle_c.schedule(abi.default_profile(), s.cluster, s.pods, n_pods, s.n_nodes, record="meta",
                                      threads=min(16, os.cpu_count() or 1), n_classes=s.cluster.n_classes,
                                      n_terms=s.cluster.n_terms)
    nc = s.cluster.n_classes
    cls = np.array([s.pods.pods[j].cls for j in range(n_pods)])
    assert all(s.pods.pods[j].own_terms_len == 0 for j in range(n_pods))  # class rows only (C4 recipe)
    # the loaded counts, read from the cluster arrays (no extra context: the allocation
    # sequence stays the product test's)
    init_cc = np.ctypeslib.as_array(s.cluster.class_count, shape=(nc * n_nodes,)).reshape(nc, n_nodes).astype(np.int64)
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)
    W = 2 * wl
    first = None
    for rep in range(runs):
        findings = []
        sp.reset()
        outs = sp.run(n_pods)
        bad = [np.flatnonzero(np.asarray(ch) != ch_o) for ch in outs]
        assert sp.ctxs[0].last_timing()[1] == 2 * -(-n_pods // per_chunk)  # as the product test
        g = sp.node_state()
        cc_bad = np.argwhere(g["class_count"][:nc, :n_nodes] != st["class_count"][:nc, :n_nodes])
        print(f"run {rep}: mismatching pods {[b.tolist()[:6] for b in bad]}; final class counts differing from the "
              f"oracle (class, node, device, oracle) "
              f"{[(int(a), int(b), int(g['class_count'][a, b]), int(st['class_count'][a, b])) for a, b in cc_bad[:8]]}")
        tr = [_fetch(c, n_pods, W) for c in sp.ctxs]
        for p, (words, lst, rows) in enumerate(tr):
            lo, hi = split.part_rows(n_nodes, 2, wl, p)
            own = slice(p * wl, (p + 1) * wl)
            w = words[:, own]
            chosen = np.asarray(outs[p])
            exp = _replay(cls, chosen, init_cc, n_pods)
            for name in ("REREAD", "BAD_ST", "BAD_REC", "BAD_LBL", "PRO"):
                hit = np.argwhere(w[:, :, GT[name]] != 0)
                if len(hit):
                    findings.append(f"run {rep} part {p} {name} at (pod, shard, value) "
                                    f"{[(int(a), int(b) + p * wl, int(w[a, b, GT[name]])) for a, b in hit[:10]]}")
            findings += _check_list(f"run {rep} part {p}", lst, exp, rows, lo, hi, per_chunk, n_pods)
            for k in range(n_pods):  # the winner's count before its commit
                x = int(chosen[k])
                if x < lo or x >= hi:
                    continue
                ws = [j for j in range(wl) if w[k, j, GT["CMT"]] > 0]
                if len(ws) != 1:
                    findings.append(f"run {rep} part {p} pod {k}: commit recorded by shards {ws}")
                    continue
                r = w[k, ws[0]]
                before = int(r[GT["CMT"] + 2])
                want = exp[k].get((int(cls[k]), x), 0)
                if before >= 0 and before != want:
                    findings.append(f"run {rep} part {p} pod {k} (class {int(cls[k])}) on node {x}: count before the "
                                    f"commit {before}, replay {want}")
            if first is not None:
                dl = np.argwhere((first[p][:, own, :32] != w[:, :, :32]).any(axis=2))
                if len(dl):
                    findings.append(f"run {rep} part {p} local bins differing from run 0 at (pod, shard) "
                                    f"{[(int(a), int(b) + p * wl) for a, b in dl[:10]]}")
        if first is None:
            first = [t[0].copy() for t in tr]
        for f in findings[:40]:
            print("  ", f)
    sp.close()
