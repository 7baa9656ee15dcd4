"""A/B of the per-pod service grid (kss_service_eval + kss_service_commit) under kss_set_option
settings (not part of the product path).

    python tools/ab_service.py CONFIG N_PODS "opt=v,..." ["opt=v,..." ...]

Per setting: the C<CONFIG> cluster (the bench's sizes and seed), N_PODS staged pods, one warm-up
pass, then one timed pass of eval + commit per pod with every field (full record) and one with
the slim fields; prints the median eval us of each and whether the chosen nodes equal the first
setting's (a parity smoke: tests/test_gpu_service.py holds the parity tests)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kube-scheduler-simulator_amd"))

import numpy as np  # noqa: E402

from kss import abi, native  # noqa: E402
from kss.synth import SEED_BASE  # noqa: E402

SIZES = {1: 100, 2: 5000, 3: 5000}


def main():
    cfg, n_pods = int(sys.argv[1]), int(sys.argv[2])
    settings = sys.argv[3:] or [""]
    s = native.Synth(cfg, SEED_BASE + cfg, SIZES[cfg], n_pods)
    ref = None
    slim = abi.KSS_FIELD_FAIL | abi.KSS_FIELD_DETAIL | abi.KSS_FIELD_TOTAL
    for setting in settings:
        native.reset_options()
        for kv in filter(None, setting.split(",")):
            k, v = kv.split("=")
            native.set_option(k, int(v))
        ctx = native.Context(abi.default_profile())
        ctx.load(s.cluster)
        ctx.stage(s.pods)
        view = abi.PodView()
        res = {}
        for fields, name in ((abi.KSS_FIELD_ALL, "full"), (slim, "slim")):
            for rep in range(2):  # warm-up, then timed
                ctx.reset()
                ev, ch = [], []
                for j in range(n_pods):
                    a = time.perf_counter()
                    native.check(native.lib().kss_service_eval(ctx.h, j, fields, ctypes.byref(view)))
                    ev.append(time.perf_counter() - a)
                    ch.append(view.chosen)
                    if view.chosen >= 0:
                        native.check(native.lib().kss_service_commit(ctx.h, j, view.chosen))
                ctx.service_stop()
            res[name] = float(np.median(ev) * 1e6)
            ref = ch if ref is None else ref
            res[name + "_same"] = ch == ref
        print(f"C{cfg} [{setting or 'default'}] mode {ctx.service_mode()} full {res['full']:.1f} us "
              f"slim {res['slim']:.1f} us same_as_first={res['full_same'] and res['slim_same']}", flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
