#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel mean duration and the mean
gap before each kernel (previous kernel end -> this kernel start) on its queue.
    python scripts/trace_timeline.py gpurun_out/x/run_kernel_trace.csv [last_n]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-last:]
    dur = defaultdict(list)
    gap = defaultdict(list)
    prev_end = None
    for r in rows:
        k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][-60:]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[k].append(e - s)
        if prev_end is not None:
            gap[k].append(s - prev_end)
        prev_end = e
    for k in sorted(dur, key=lambda x: -sum(dur[x])):
        d, g = dur[k], gap[k]
        print(f"{k:62s} n={len(d):6d} mean {sum(d) / len(d) / 1e3:8.2f} us  gap-before {sum(g) / max(len(g), 1) / 1e3:8.2f} us")


if __name__ == "__main__":
    main()
