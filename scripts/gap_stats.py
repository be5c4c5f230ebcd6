#!/usr/bin/env python3
"""Gaps between consecutive kernels on the GPU timeline of a rocprofv3
--kernel-trace run (kernel_trace.csv): where the time between the round
kernels goes.  Prints a histogram of the gaps and the largest ones with the
kernels on either side."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows))
# the timed region: from the last "warmup" boundary, take the last 40 % of the run
ks = ks[int(len(ks) * 0.6):]
gaps = []
for a, b in zip(ks, ks[1:]):
    gaps.append((b[0] - a[1], a[2], b[2]))
busy = sum(e - s for s, e, _ in ks)
span = ks[-1][1] - ks[0][0]
print(f"kernels {len(ks)}, span {span/1e6:.2f} ms, busy {busy/1e6:.2f} ms, idle {(span-busy)/1e6:.2f} ms")
edges = [0, 500, 1000, 2000, 4000, 8000, 16000, 50000, 1e12]
for lo, hi in zip(edges, edges[1:]):
    sel = [g for g, _, _ in gaps if lo <= g < hi]
    print(f"  gap {lo/1e3:7.1f}-{hi/1e3:7.1f} us: {len(sel):6d}  total {sum(sel)/1e6:8.3f} ms")
print("largest gaps:")
for g, a, b in sorted(gaps, reverse=True)[:12]:
    print(f"  {g/1e3:9.1f} us  after {a}  before {b}")
