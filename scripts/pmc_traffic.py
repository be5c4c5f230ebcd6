#!/usr/bin/env python3
"""HBM bytes per round of the round kernel over bench.py's timed region, from
separate rocprofv3 FETCH_SIZE and WRITE_SIZE passes of the same bench command
(each pass's own bench JSON line gives its timed batches and rounds), with the
FETCH_SIZE correction measured by scripts/pmc_calib.py:

    python3 scripts/pmc_traffic.py <fetch dir> <write dir> <fetch bench JSON> <write bench JSON> \
        <calibration JSON> --key c3-10000h/k_round_ps [--out profiles/r03/pmc_traffic.json]

The timed region's dispatches are the kernel's last `timed_batches` dispatches
(bench.py runs nothing after its timed region but the summary); the bytes are
summed over them and divided by the timed rounds.  The entry is written under
`key` (bench.py's roofline.traffic_key: workload and kernel), with the SHA-1 of
the engine source it was taken of; bench.py reads it only for that source.
"""
import argparse
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "shadow-1_amd"))


def per_dispatch(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    key = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(vals))
                    vals.append((key, float(row["Counter_Value"]) * 1024.0))   # KB -> B
    vals.sort()
    # one row per (dispatch, counter): sum the per-XCD / per-instance rows of a dispatch
    out = {}
    for k, v in vals:
        out[k] = out.get(k, 0.0) + v
    return [out[k] for k in sorted(out)]


def bench_line(path):
    return json.loads([l for l in open(path).read().splitlines() if l.strip().startswith("{")][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("fetch_bench")
    ap.add_argument("write_bench")
    ap.add_argument("calibration")
    ap.add_argument("--key", required=True)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "pmc_traffic.json"))
    a = ap.parse_args()
    kernel = a.key.split("/")[1]
    cal = json.load(open(a.calibration))
    corr = float(cal["read_correction"])
    res = {}
    for name, d, counter, bj in (("fetch", a.fetch_dir, "FETCH_SIZE", a.fetch_bench),
                                 ("write", a.write_dir, "WRITE_SIZE", a.write_bench)):
        vals = per_dispatch(d, counter, kernel)
        b = bench_line(bj)
        nb = int(b.get("timed_batches") or 0)
        rounds = int(b.get("rounds") or 0)
        if b["roofline"]["kernel"] != kernel or not nb or nb > len(vals):
            raise SystemExit(f"{name}: kernel {b['roofline']['kernel']} / {nb} timed batches vs {len(vals)} dispatches")
        res[name] = {"dispatches": len(vals), "timed_dispatches": nb, "timed_rounds": rounds,
                     "bytes_timed": sum(vals[-nb:]), "per_round": sum(vals[-nb:]) / rounds,
                     "alg_bytes_per_round": b["roofline"]["bytes_per_launch"]}
    read = res["fetch"]["per_round"] * corr
    write = res["write"]["per_round"]
    alg = res["fetch"]["alg_bytes_per_round"]
    import shdgpu as S
    ent = {"hbm_bytes_per_round": round(read + write, 1), "read_bytes_per_round": round(read, 1),
           "write_bytes_per_round": round(write, 1), "fetch_correction": corr,
           "fetch_correction_source": "scripts/pmc_calib.py (k_rec_read: 128-B records, one lane per host, 8 x 16 B)",
           "alg_bytes_per_round": alg, "traffic_over_alg": round((read + write) / alg, 3) if alg else None,
           "passes": res}
    prof = {}
    if os.path.exists(a.out):
        prof = json.load(open(a.out))
    sha = S.engine_source_sha1()
    if prof.get("engine_source_sha1") != sha:
        prof = {"engine_source_sha1": sha, "entries": {}}
    prof["entries"][a.key] = ent
    with open(a.out, "w") as f:
        json.dump(prof, f, indent=1)
    print(json.dumps({a.key: {k: ent[k] for k in ("hbm_bytes_per_round", "alg_bytes_per_round", "traffic_over_alg")}}))


if __name__ == "__main__":
    main()
