"""Diagnosis of a nondeterministic result: repeat one scheduling scenario and count the runs
whose chosen vector differs from the C oracle's.  Modes:
  split   InProcessSplit(2 parts x wl shards) over KSS_STATIC_BYTES-forced chunks
  single  one context, KSS_SHARDS = 2 * wl shards, the same chunks (no split grid)
usage: python tools/diag_flake.py MODE [reps] [config n_nodes n_pods per_chunk wl]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("kube-scheduler-simulator_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))

import numpy as np  # noqa: E402


def main():
    mode = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    config, n_nodes, n_pods, per_chunk, wl = (int(x) for x in (sys.argv[3:8] if len(sys.argv) > 7 else (4, 6000, 200, 24, 16)))
    os.environ["KSS_STATIC_BYTES"] = str(4 * n_nodes * per_chunk)
    if mode == "single":
        os.environ["KSS_SHARDS"] = str(2 * wl)
    import torch
    torch.zeros(1, device="cuda")
    import oracle_c
    from kss import abi, native, split
    from kss.synth import SEED_BASE
    s = native.Synth(config, SEED_BASE + config, n_nodes, n_pods)
    ch_o, _, _ = oracle_c.schedule(abi.default_profile(), s.cluster, s.pods, n_pods, s.n_nodes, record="meta",
                                   threads=16, n_classes=s.cluster.n_classes, n_terms=s.cluster.n_terms)
    if mode == "split":
        sp = split.InProcessSplit(s.cluster, s.pods, 2, wl)
        reset, run = sp.reset, lambda: sp.run(n_pods)
    else:
        ctx = native.Context(abi.default_profile())
        ctx.load(s.cluster)
        ctx.stage(s.pods)
        reset, run = ctx.reset, lambda: [ctx.run_staged(n_pods)]
    bad = 0
    for r in range(reps):
        reset()
        t0 = time.perf_counter()
        outs = run()
        diffs = [np.flatnonzero(np.asarray(ch) != ch_o) for ch in outs]
        nd = [len(d) for d in diffs]
        bad += any(nd)
        first = [int(d[0]) if len(d) else -1 for d in diffs]
        print(f"{mode} rep {r}: mismatches per part {nd} first pod {first} ({time.perf_counter() - t0:.2f} s)", flush=True)
        if any(nd) and bad == 1:  # the first bad run: what the device returned
            ctxs = sp.ctxs if mode == "split" else [ctx]
            for p, (ch, cx) in enumerate(zip(outs, ctxs)):
                j = first[p] if first[p] >= 0 else 0
                print(f"  part {p}: chosen[:8] {np.asarray(ch)[:8].tolist()} oracle {ch_o[:8].tolist()}; "
                      f"meta[{j}] {cx.fetch_meta(n_pods)[j].tolist()} kernel {cx.last_kernel()} timing {cx.last_timing()}",
                      flush=True)
    print(f"{mode}: {bad} of {reps} runs differ from the oracle", flush=True)


if __name__ == "__main__":
    main()
