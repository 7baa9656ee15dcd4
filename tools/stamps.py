"""Summarise KSS_STAMPS_FILE dumps: median per-phase durations (µs) of the first pods of each launch.
Phases: 0 pod start, 1 plan, 2 filter pass done, 3 filter exchange done, 4 normalize pass done,
5 argmax exchange done, 6 commit + barrier done."""
import sys

import numpy as np

NAMES = ["plan", "filter", "x_filter", "normalize", "x_argmax", "commit"]
# k_simple: 0 start, 1 pass B, 2 best-key reduction, 3 pass A, 4 statistics reduction,
# 5 exchange + barrier, 6 commit + ring store
NAMES_SIMPLE = ["passB", "red_best", "passA", "red_stats", "xchg", "commit"]


def summarise_simple(path):
    """k_simple records 16 stamps per pod: 0..6 the loop phases, 7 eval start (lane 0 of
    shard 0, first slot), 8 filters done, 9 TT+NA scores, 10 Fit score, 11 BA score."""
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    a = a[(a[:, 0] > 0) & (a[:, 6] > 0)]
    d = np.diff(a[:, :7], axis=1) / 100.0
    out = " ".join(f"{n}={m:.2f}" for n, m in zip(NAMES_SIMPLE, np.median(d, axis=0)))
    e = a[a[:, 11] > 0]
    if len(e):
        sub = {"filters": (7, 8), "tt_na": (8, 9), "fit": (9, 10), "ba": (10, 11), "after_eval": (11, 3)}
        out += " || " + " ".join(f"{k}={np.median(e[:, j] - e[:, i]) / 100.0:.2f}" for k, (i, j) in sub.items())
    tot = (a[:, 6] - a[:, 0]) / 100.0
    return out + f" | pod={np.median(tot):.2f} us (n={len(a)})"


def summarise(path):
    if "simple" in path:
        return summarise_simple(path)
    names = NAMES
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    a = a[(a[:, 0] > 0) & (a[:, 6] > 0)]
    d = np.diff(a[:, :7].astype(np.int64), axis=1) / 100.0  # 100 MHz -> µs
    tot = (a[:, 6].astype(np.int64) - a[:, 0].astype(np.int64)) / 100.0
    med = np.median(d, axis=0)
    return " ".join(f"{n}={m:.2f}" for n, m in zip(names, med)) + f" | pod={np.median(tot):.2f} us (n={len(a)})"


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p, summarise(p))
