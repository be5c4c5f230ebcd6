#!/usr/bin/env python3
"""k_tcp_round per-dispatch durations from rocprofv3 kernel traces (one
directory per variant): count, total, median and the slowest 12 dispatches
(the rounds where the bench model's connections start).
    python3 scripts/r04/tcp_dispatch.py DIR_A DIR_B ..."""
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_tcp_round" in r["Kernel_Name"]]
    top = sorted(us, reverse=True)[:12]
    print(f"{d}: k_tcp_round dispatches {len(us)}, total {sum(us) / 1e3:.1f} ms, median {statistics.median(us):.0f} us, "
          f"slowest 12 (us) {[round(x) for x in top]}, their sum {sum(top) / 1e3:.1f} ms")
