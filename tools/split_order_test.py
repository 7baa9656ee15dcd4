"""Experiment (not part of the suite): the many-chunk split scenario of
tests/test_gpu_split.py::test_parts_over_many_chunks[4-6000-200-24-16] with the parts'
threads started in reverse order (part 1 first), reporting every count word that differs
from the oracle after each run and which part owns it.  Run in the position of the suite's
test (after the spread / split tests), product library:

    python -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py \\
        tests/test_gpu_split.py::test_in_process_parts_match_oracle \\
        "tests/test_gpu_split.py::test_parts_over_many_chunks[2-3000-240-30-8]" \\
        "tests/test_gpu_split.py::test_parts_over_many_chunks[2-3000-240-31-8]" \\
        tools/split_order_test.py -m gpu -k 'spread or split or in_process or many_chunks or order' -s
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(ROOT, "kube-scheduler-simulator_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
import oracle_c  # noqa: E402
from kss import abi, native, split  # noqa: E402
from kss.synth import SEED_BASE  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("order", ["reversed"])
def test_order_many_chunks(monkeypatch, order):
    config, n_nodes, n_pods, per_chunk, wl = 4, 6000, 200, 24, 16
    monkeypatch.setenv("KSS_STATIC_BYTES", str(4 * n_nodes * per_chunk))
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, res, st = oracle_c.schedule(abi.default_profile(), s.cluster, s.pods, n_pods, s.n_nodes, record="meta",
                                      threads=min(16, os.cpu_count() or 1), n_classes=s.cluster.n_classes,
                                      n_terms=s.cluster.n_terms)
    sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)
    nc = s.cluster.n_classes
    lo1, _ = split.part_rows(n_nodes, 2, wl, 1)
    bad_runs = 0
    for rep in range(3):
        sp.reset()
        fns = [lambda c=c: c.run_staged(n_pods) for c in sp.ctxs]
        outs = split._run_concurrently(fns[::-1])[::-1] if order == "reversed" else split._run_concurrently(fns)
        bad = [np.flatnonzero(np.asarray(ch) != ch_o).tolist()[:6] for ch in outs]
        g = sp.node_state()
        d = np.argwhere(g["class_count"][:nc, :n_nodes] != st["class_count"][:nc, :n_nodes])
        words = [(int(a), int(b), "part 1" if b >= lo1 else "part 0", int(g["class_count"][a, b]),
                  int(st["class_count"][a, b])) for a, b in d[:8]]
        print(f"{order} run {rep}: mismatching pods {bad}; class counts differing (class, node, owner, device, "
              f"oracle) {words}")
        bad_runs += bool(len(d)) or any(bad)
    sp.close()
    assert not bad_runs
