"""Probe for the many-chunk split flake (tests/test_gpu_split.py::test_parts_over_many_chunks
[4-6000-200-24-16], seen only after other GPU tests ran in the same process): the same
scenario repeated as a split grid, as one context with the same shards and chunks, and as a
split grid without chunking, printing each run's mismatches against the C oracle.  Always
passes; run after the modules that reproduce it, e.g.
  python -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tools/flake_probe_test.py -m gpu -s -q"""
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


def _report(tag, rep, outs, ch_o, ctxs, n_pods):
    bad = [np.flatnonzero(np.asarray(ch) != ch_o) for ch in outs]
    if not any(len(b) for b in bad):
        print(f"{tag} run {rep}: ok", flush=True)
        return 0
    j = int(next(b for b in bad if len(b))[0])
    meta = [c.fetch_meta(n_pods)[j].tolist() for c in ctxs]
    print(f"{tag} run {rep}: mismatching {[b.tolist()[:6] for b in bad]} first {j}: device "
          f"{[int(o[j]) for o in outs]} meta {meta} oracle {int(ch_o[j])}", flush=True)
    return 1


def test_probe(monkeypatch):
    config, n_nodes, n_pods, per_chunk, wl = 4, 6000, 200, 24, 16
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, _, _ = oracle_c.schedule(abi.default_profile(), s.cluster, s.pods, n_pods, s.n_nodes, record="meta",
                                   threads=16, n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    monkeypatch.setenv("KSS_STATIC_BYTES", str(4 * n_nodes * per_chunk))
    bad = {}
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)
    bad["split_chunks"] = 0
    for rep in range(6):
        sp.reset()
        bad["split_chunks"] += _report("split chunks", rep, sp.run(n_pods), ch_o, sp.ctxs, n_pods)
    sp.close()
    monkeypatch.setenv("KSS_SHARDS", str(2 * wl))
    ctx = native.Context(abi.default_profile())
    ctx.load(s.cluster)
    ctx.stage(s.pods)
    bad["single_chunks"] = 0
    for rep in range(6):
        ctx.reset()
        bad["single_chunks"] += _report("single chunks", rep, [ctx.run_staged(n_pods)], ch_o, [ctx], n_pods)
    ctx.close()
    monkeypatch.delenv("KSS_SHARDS")
    monkeypatch.delenv("KSS_STATIC_BYTES")
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)
    bad["split_one_chunk"] = 0
    for rep in range(4):
        sp.reset()
        bad["split_one_chunk"] += _report("split one chunk", rep, sp.run(n_pods), ch_o, sp.ctxs, n_pods)
    sp.close()
    print("probe summary (runs with mismatches):", bad, flush=True)
