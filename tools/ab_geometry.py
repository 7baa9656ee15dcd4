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


def main():
    cfg = int(sys.argv[1])
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
