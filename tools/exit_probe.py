"""Exit-crash probe under rocprofv3: the bench's GPU sequence without the bench itself."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-scheduler-simulator_amd"))
from kss import abi, native  # noqa: E402

step = sys.argv[1] if len(sys.argv) > 1 else "all"
s = native.Synth(2, 0x5EED0002, 5000, 10000)
ctx = native.Context(abi.default_profile())
ctx.load(s.cluster)
ctx.stage(s.pods)
for _ in range(2):
    ctx.reset()
    ctx.run_staged(10000)
print(ctx.last_timing(), ctx.last_geometry(), ctx.last_kernel())
if step in ("all", "close"):
    ctx.close()
    s.close()
print("done", flush=True)
