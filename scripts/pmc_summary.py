#!/usr/bin/env python3
"""Mean per-dispatch SQ counters of one kernel from rocprofv3 --pmc CSV output.

    python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 [--kernel k_round_dev]

Prints each counter's mean over the kernel's dispatches, and per-wave ratios
when SQ_WAVES is present (instructions per wave, cycles per instruction).
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_round_dev")
    a = ap.parse_args()
    vals = defaultdict(list)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if a.kernel in row["Kernel_Name"]:
                        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in vals.items()}
    for k in sorted(mean):
        print(f"{k:24s} {mean[k]:16.1f}  ({len(vals[k])} dispatches)")
    w = mean.get("SQ_WAVES")
    if w:
        print(f"per wave ({w:.0f} waves/dispatch):")
        for k in sorted(mean):
            if k.startswith("SQ_INSTS") or k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE") or k == "SQ_WAVE_CYCLES":
                print(f"  {k:22s} {mean[k] / w:12.1f}")
        insts = sum(mean.get(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                                             "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"))
        if insts and "SQ_WAVE_CYCLES" in mean:
            print(f"  instructions/wave {insts / w:.0f} (of the counted kinds); wave cycles per instruction "
                  f"{mean['SQ_WAVE_CYCLES'] / insts:.1f}")


if __name__ == "__main__":
    main()
