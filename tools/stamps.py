"""Summarise KSS_STAMPS_FILE dumps: median per-phase durations (µs) of the first pods of each launch.
Phases: 0 pod start, 1 plan, 2 filter pass done, 3 filter exchange done, 4 normalize pass done,
5 argmax exchange done, 6 commit + barrier done."""
import sys

import numpy as np

NAMES = ["plan", "filter", "x_filter", "normalize", "x_argmax", "commit"]


def summarise(path):
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    a = a[(a[:, 0] > 0) & (a[:, 6] > 0)]
    d = np.diff(a[:, :7].astype(np.int64), axis=1) / 100.0  # 100 MHz -> µs
    tot = (a[:, 6].astype(np.int64) - a[:, 0].astype(np.int64)) / 100.0
    med = np.median(d, axis=0)
    return " ".join(f"{n}={m:.2f}" for n, m in zip(NAMES, med)) + f" | pod={np.median(tot):.2f} us (n={len(a)})"


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p, summarise(p))
