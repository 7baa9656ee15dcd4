import os, sys
sys.path.insert(0, "kube-scheduler-simulator_amd")
from kss import abi, native
native.set_stamps_file("gpurun_out/c2.stamps")
from kss.synth import DEFAULT_SIZES, SEED_BASE
s = native.Synth(2, SEED_BASE + 2, DEFAULT_SIZES[2][0], 1000)
ctx = native.Context(abi.default_profile(), device=0)
ctx.load(s.cluster); ctx.stage(s.pods); ctx.run_staged(s.n_pods)
print(ctx.last_geometry())
ctx.close(); s.close()
