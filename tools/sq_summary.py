"""Summarise rocprofv3 --pmc passes (gpurecipe.sh sq_* steps) per kernel.

    python tools/sq_summary.py gpurun_out/r5k_sq_c2_pmc0 gpurun_out/r5k_sq_c2_pmc1 ... > profiles/x.txt

Every pass's p_counter_collection.csv holds one row per (dispatch, counter).  Printed per
kernel whose name contains --kernel (default k_simple): dispatches, the mean value per
dispatch of every counter collected, and the derived ratios the DESIGN tables quote
(VALU instructions per wave, issue-busy fractions of SQ_WAVE_CYCLES / SQ_BUSY_CYCLES)."""
import argparse
import csv
import os
from collections import defaultdict


def load(dirs, pattern):
    vals = defaultdict(list)  # counter -> values per dispatch
    names = set()
    for d in dirs:
        f = os.path.join(d, "p_counter_collection.csv")
        if not os.path.exists(f):
            continue
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if pattern not in row["Kernel_Name"]:
                    continue
                names.add(row["Kernel_Name"])
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return names, vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_simple")
    a = ap.parse_args()
    names, vals = load(a.dirs, a.kernel)
    if not vals:
        print(f"no dispatch of a kernel matching {a.kernel!r}")
        return
    for n in sorted(names):
        print("kernel:", n)
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    print(f"{'counter':28s} {'dispatches':>10s} {'mean per dispatch':>20s}")
    for k in sorted(mean):
        print(f"{k:28s} {len(vals[k]):10d} {mean[k]:20.1f}")
    waves = mean.get("SQ_WAVES")
    print("derived:")
    if waves:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH"):
            if k in mean:
                print(f"  {k + ' per wave':34s} {mean[k] / waves:14.1f}")
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC"):
            if k in mean:
                print(f"  {k + ' / SQ_WAVE_CYCLES':44s} {mean[k] / wc:8.3f}")
    if "GRBM_GUI_ACTIVE" in mean and "SQ_BUSY_CYCLES" in mean:
        print(f"  {'SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE':44s} {mean['SQ_BUSY_CYCLES'] / mean['GRBM_GUI_ACTIVE']:8.3f}")


if __name__ == "__main__":
    main()
