"""Probe 2 for the many-chunk split flake: the scenario of
tests/test_gpu_split.py::test_parts_over_many_chunks[4-6000-200-24-16] with KSS_SPREAD_DEBUG,
three runs; for every pod whose choice differs from the oracle, the shards whose local
statistics bins (or whose exchanged bins / minima) differ from the first run's are printed.
Run after the modules that reproduce the failure:
  python -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py \\
      tools/flake_probe2_test.py -m gpu -k "spread or split or probe" -s -q"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("kube-scheduler-simulator_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402
import pytest  # noqa: E402

import oracle_c  # noqa: E402
from kss import abi, native, split  # noqa: E402
from kss.synth import SEED_BASE  # noqa: E402

pytestmark = pytest.mark.gpu


def _dump(ctx, n, W):
    out = np.zeros(n * W * 64, np.int32)
    k = native.lib().kss_debug_spread(ctx.h, out.ctypes.data_as(C.POINTER(C.c_int32)), out.size)
    assert k == out.size, k
    return out.reshape(n, W, 64)


def test_probe_split_debug(monkeypatch):
    config, n_nodes, n_pods, per_chunk, wl = 4, 6000, 200, 24, 16
    W = 2 * wl
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, _, _ = oracle_c.schedule(abi.default_profile(), s.cluster, s.pods, n_pods, s.n_nodes, record="meta",
                                   threads=16, n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    monkeypatch.setenv("KSS_STATIC_BYTES", str(4 * n_nodes * per_chunk))
    monkeypatch.setenv("KSS_SPREAD_DEBUG", "1")
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)
    dumps, outs_all = [], []
    for rep in range(4):
        sp.reset()
        outs = sp.run(n_pods)
        outs_all.append(outs)
        d = [_dump(c, n_pods, W) for c in sp.ctxs]
        # each part wrote its own shards' rows: merge (part p: shards [p * wl, (p + 1) * wl))
        m = d[0].copy()
        m[:, wl:, :] = d[1][:, wl:, :]
        dumps.append((m, d))
        bad = [np.flatnonzero(np.asarray(ch) != ch_o) for ch in outs]
        print(f"run {rep}: mismatches {[b.tolist()[:6] for b in bad]}", flush=True)
    sp.close()
    ref = dumps[0][0]
    for rep in range(1, 4):
        m, d = dumps[rep]
        pods = sorted(set(np.flatnonzero(np.asarray(outs_all[rep][0]) != ch_o).tolist()))
        for j in pods[:2]:
            diff_local = [(w, int(b), int(ref[j, w, b]), int(m[j, w, b])) for w in range(W) for b in range(26)
                          if ref[j, w, b] != m[j, w, b]]
            diff_glob = [(p, w, int(b), int(ref[j, w, b]), int(d[p][j, w, b])) for p in range(2)
                         for w in range(p * wl, (p + 1) * wl) for b in range(32, 63) if ref[j, w, b] != d[p][j, w, b]]
            print(f"run {rep} pod {j}: local bins differing (shard, bin, run0, now) {diff_local[:12]}", flush=True)
            print(f"run {rep} pod {j}: exchanged values differing (part, shard, slot, run0, now) {diff_glob[:12]}",
                  flush=True)
            print(f"run {rep} pod {j}: epochs {sorted(set(m[j, :, 63].tolist()))} run0 {sorted(set(ref[j, :, 63].tolist()))}",
                  flush=True)
    # the previous pods too: the first pod (of any run) whose local bins differ from run 0
    for rep in range(1, 4):
        m = dumps[rep][0]
        diff = np.flatnonzero((m[:, :, :26] != ref[:, :, :26]).any(axis=(1, 2)))
        print(f"run {rep}: pods whose local bins differ from run 0: {diff.tolist()[:10]}", flush=True)
