"""A/B of k_simple / k_spread geometries through kss_set_option (not part of the product path).

    python tools/ab_geometry.py CONFIG "opt=v,opt=v" ["opt=v,..." ...]

Per setting: one C<CONFIG> batch (BASELINE recipe and seed, the bench's sizes) staged once, one
warm-up run and three timed runs of the whole sequential batch; prints the geometry, the kernel,
pods/s and whether the chosen nodes equal the first setting's (a parity smoke, not a parity test:
tests/ hold those).  An empty string is the default geometry."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-scheduler-simulator_amd"))

import numpy as np  # noqa: E402

from kss import abi, native  # noqa: E402
from kss.synth import SEED_BASE  # noqa: E402

SIZES = {1: (100, 1000), 2: (5000, 10000), 3: (5000, 10000), 4: (100000, 20000)}


def sweep_ab(settings):
    """C5 shape: 512 scenarios x 1,000 nodes x 1,000 pods in one resident sweep, per setting."""
    n_scen = int(os.environ.get("AB_SCEN", "512"))
    syn = [native.Synth(5, SEED_BASE + 5 + 7919 * k, 1000, 1000) for k in range(n_scen)]
    ref = None
    for setting in settings or [""]:
        native.reset_options()
        for kv in filter(None, setting.split(",")):
            k, v = kv.split("=")
            native.set_option(k, int(v))
        sw = native.Sweep(abi.default_profile(), [x.cluster for x in syn], [x.pods for x in syn])
        sw.run()
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            chosen, ms = sw.run()
            wall = time.perf_counter() - t0
            best = wall if best is None else min(best, wall)
        same = ref is None or bool(np.array_equal(chosen, ref))
        ref = chosen if ref is None else ref
        print(f"C5 x{n_scen} [{setting or 'default'}] {sw.info()['kernel']} {n_scen * 1e6 / best / 1e9:.2f} G evals/s "
              f"({best * 1e3:.2f} ms) same_as_first={same}", flush=True)
        sw.close()
    native.reset_options()


def main():
    cfg = int(sys.argv[1])
    if cfg == 5:
        return sweep_ab(sys.argv[2:])
    n_nodes, n_pods = SIZES[cfg]
    pct = int(os.environ.get("AB_PCT", "100"))
    s = native.Synth(cfg, SEED_BASE + cfg, n_nodes, n_pods)
    ref = None
    for setting in sys.argv[2:] or [""]:
        native.reset_options()
        for kv in filter(None, setting.split(",")):
            k, v = kv.split("=")
            native.set_option(k, int(v))
        prof = abi.default_profile()
        prof.pct_nodes_to_score = pct
        ctx = native.Context(prof)
        ctx.load(s.cluster)
        ctx.stage(s.pods)
        ctx.reset()
        ctx.run_staged(n_pods)
        ts = []
        for _ in range(3):
            ctx.reset()
            t0 = time.perf_counter()
            chosen = ctx.run_staged(n_pods)
            ts.append(time.perf_counter() - t0)
        same = ref is None or bool(np.array_equal(chosen, ref))
        ref = chosen if ref is None else ref
        print(f"C{cfg} pct={pct} [{setting or 'default'}] {ctx.last_kernel()} {ctx.last_geometry()} "
              f"{n_pods / min(ts):.0f} pods/s ({min(ts) / n_pods * 1e6:.2f} us/pod) same_as_first={same}", flush=True)
        ctx.close()
    native.reset_options()
    s.close()


if __name__ == "__main__":
    main()
