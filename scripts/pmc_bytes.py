#!/usr/bin/env python3
"""HBM bytes per dispatch of the round kernel from the rocprofv3 FETCH_SIZE
and WRITE_SIZE passes of scripts/profile_round.sh, written as
profiles/r01/k_round_pmc_bytes.json (read by bench.py's roofline `traffic`
when the profiled engine source matches the one being run).

    python scripts/pmc_bytes.py gpurun_out/prof_fetch gpurun_out/prof_write [--kernel k_round_tl]

FETCH_SIZE is doubled: gfx950 reports half of the bytes of 16-B-per-lane
reads (MI355X_MICROARCH.md, HBM / rocprofv3 section); WRITE_SIZE as read.
Both counters are in KB.
"""
import argparse
import csv
import glob
import hashlib
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter, kernel):
    """the counter's value per dispatch of `kernel`, in dispatch order"""
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    key = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(vals))
                    vals.append((key, float(row["Counter_Value"])))
    return [v for _, v in sorted(vals)]


def timed(vals, bench_json):
    """the timed region's dispatches: the last 64 x (ticketless batches) of
    the run (bench.py --pmc-run writes the counts of its timed region); None
    unless every timed batch was ticketless"""
    try:
        b = json.load(open(bench_json))
    except (OSError, ValueError):
        return None
    n = int(b.get("timed_batches_ticketless") or 0) * 64
    if not n or int(b.get("timed_batches") or -1) * 64 != n or n > len(vals):
        return None
    return vals[-n:], int(b["rounds"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--kernel", default="k_round_tl")
    ap.add_argument("--fetch-bench", help="the FETCH_SIZE pass's bench.py JSON line (its timed-region counts)")
    ap.add_argument("--write-bench", help="the WRITE_SIZE pass's bench.py JSON line")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r02", "k_round_pmc_bytes.json"))
    a = ap.parse_args()
    fe = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    wr = per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel)
    if not fe or not wr:
        raise SystemExit(f"no {a.kernel} dispatches with FETCH_SIZE / WRITE_SIZE")
    f_kb = sum(fe) / len(fe)
    w_kb = sum(wr) / len(wr)
    src = open(os.path.join(REPO, "shadow-1_amd", "csrc", "engine.hip"), "rb").read()
    out = {
        "kernel": a.kernel,
        "FETCH_SIZE_KB_avg_per_dispatch": round(f_kb, 3),
        "FETCH_SIZE_dispatches": len(fe),
        "WRITE_SIZE_KB_avg_per_dispatch": round(w_kb, 3),
        "WRITE_SIZE_dispatches": len(wr),
        "hbm_bytes_per_dispatch": int(round((2 * f_kb + w_kb) * 1024)),
        "correction": "FETCH_SIZE doubled (gfx950 reports 1/2 of 16-B/lane reads, MI355X_MICROARCH.md "
                      "HBM/rocprofv3 section); WRITE_SIZE as read",
        "command": "rocprofv3 --pmc FETCH_SIZE (resp. WRITE_SIZE) -- python3 bench.py --steps 2 --warmup 2 --lossy-edge-loss-max 0 "
                   "--no-cpu-baseline, separate passes; averaged over every " + a.kernel + " dispatch of the run",
        "engine_source_sha1": hashlib.sha1(src).hexdigest(),
    }
    tf = timed(fe, a.fetch_bench) if a.fetch_bench else None
    tw = timed(wr, a.write_bench) if a.write_bench else None
    if tf and tw and tf[1] == tw[1]:
        # the timed region alone (warm-up rounds log first touches: halted
        # batches leave cheap forward-only launches that dilute the average):
        # the bytes of every launch of the timed batches over its rounds, as
        # bench.py's roofline counts launches
        out["timed_rounds"] = tf[1]
        out["timed_dispatches"] = len(tf[0])
        out["FETCH_SIZE_KB_timed_per_round"] = round(sum(tf[0]) / tf[1], 3)
        out["WRITE_SIZE_KB_timed_per_round"] = round(sum(tw[0]) / tw[1], 3)
        out["hbm_bytes_per_round_timed"] = int(round((2 * sum(tf[0]) + sum(tw[0])) / tf[1] * 1024))
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
