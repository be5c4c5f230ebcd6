#!/usr/bin/env python3
"""The round kernel's duration over bench.py's timed region, from a
`rocprofv3 --kernel-trace --marker-trace --output-format csv` run of bench.py
(bench.py brackets its timed region with the roctx range "shd_timed_region").

    python3 scripts/rocprof_timed.py <rocprof out dir> <bench JSON line file> [--kernel k_round_ps] [--out F]

Reports, for the dispatches of the kernel that start inside the range: their
count, total / mean / min / max duration, the span of the range, and -- with
the bench line's timed round count -- the device time per round, to set
against the line's roofline.avg_round_us (HIP events on the engine's stream,
the gaps between launches included).
"""
import argparse
import csv
import glob
import json
import os


def rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("bench_json")
    ap.add_argument("--kernel", default=None, help="kernel name substring (default: the bench line's roofline.kernel)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = [l for l in open(a.bench_json).read().splitlines() if l.strip().startswith("{")]
    bench = json.loads(lines[-1])
    kernel = a.kernel or bench["roofline"]["kernel"]
    marks = [r for r in rows(a.trace_dir, "*marker_api_trace.csv")
             if any("shd_timed_region" in str(v) for v in r.values())]
    if not marks:
        raise SystemExit("no shd_timed_region marker in the trace (run rocprofv3 with --marker-trace)")
    m = marks[-1]
    t0, t1 = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
    ks = [r for r in rows(a.trace_dir, "*kernel_trace.csv") if kernel in r["Kernel_Name"]]
    inside = [r for r in ks if t0 <= int(r["Start_Timestamp"]) <= t1]
    dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in inside]
    rounds = int(bench.get("rounds") or 0)
    out = {
        "kernel": kernel,
        "timed_region_ns": t1 - t0,
        "dispatches_in_region": len(inside),
        "dispatches_whole_run": len(ks),
        "total_ns": sum(dur),
        "mean_dispatch_us": round(sum(dur) / len(dur) / 1e3, 3) if dur else None,
        "min_dispatch_us": round(min(dur) / 1e3, 3) if dur else None,
        "max_dispatch_us": round(max(dur) / 1e3, 3) if dur else None,
        "timed_rounds": rounds,
        "device_us_per_round": round(sum(dur) / rounds / 1e3, 3) if rounds and dur else None,
        "region_us_per_round": round((t1 - t0) / rounds / 1e3, 3) if rounds else None,
        "bench_avg_round_us": bench["roofline"].get("avg_round_us", bench["roofline"].get("avg_launch_us")),
    }
    if out["device_us_per_round"] and out["bench_avg_round_us"]:
        out["bench_over_rocprof"] = round(out["bench_avg_round_us"] / out["device_us_per_round"], 4)
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
