"""Diagnosis (not a test): the 4-part in-process split grid on C4's recipe, run a few times; on a
failed final write-back check, print every part's differing words (state vs the shadow the
epilogue stored) and which buffer holds them.  python tools/final_check_probe.py [runs] [parts] [wl]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "kube-scheduler-simulator_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

torch.zeros(1, device="cuda")
from kss import native, split  # noqa: E402
from kss.synth import SEED_BASE  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
parts = int(sys.argv[2]) if len(sys.argv) > 2 else 4
wl = int(sys.argv[3]) if len(sys.argv) > 3 else 64
s = native.Synth(4, SEED_BASE + 4, 100000, 300)
sp = split.InProcessSplit(s.cluster, s.pods, parts, wl)
bad = 0
for rep in range(runs):
    sp.reset()
    try:
        sp.run(300)
        st = [c.last_handoff_status() for c in sp.ctxs]
        print(f"run {rep}: ok {st}", flush=True)
    except native.KssError as e:
        bad += 1
        print(f"run {rep}: FAILED {e}", flush=True)
        for p, c in enumerate(sp.ctxs):
            rec, entries = c.last_handoff_diag()
            print(f"  part {p}: status {c.last_handoff_status()} entries {len(entries)}", flush=True)
            for e2 in entries[:12]:
                print(f"    {e2}", flush=True)
            for e2 in entries[:3]:
                for q, c2 in enumerate(sp.ctxs):
                    for nm, (b, sz) in c2.buffer_map().items():
                        if b and b <= e2["addr"] < b + sz:
                            print(f"    word {e2['addr']:#x}: part {q} {nm} offset {e2['addr'] - b}", flush=True)
        sp.rearm()
print(f"{bad} of {runs} runs failed", flush=True)
sp.close()
