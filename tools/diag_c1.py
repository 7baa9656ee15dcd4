"""C1 diagnosis: device time and launches of one 1000-pod k_simple run."""
import sys; sys.path.insert(0, "kube-scheduler-simulator_amd")
import time

from kss import abi, native
from kss.synth import SEED_BASE

s = native.Synth(1, SEED_BASE + 1, 100, 1000)
ctx = native.Context(abi.default_profile())
ctx.load(s.cluster)
ctx.stage(s.pods)
for rep in range(3):
    ctx.reset()
    t = time.perf_counter()
    ctx.run_staged(1000)
    print("wall ms", round((time.perf_counter() - t) * 1e3, 3), "timing", ctx.last_timing(), ctx.last_kernel(), ctx.last_geometry())
