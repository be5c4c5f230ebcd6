#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE against known bytes (scripts/microbench/pmc_calib.hip):

    python3 scripts/pmc_calib.py <FETCH_SIZE pass dir> <WRITE_SIZE pass dir> <pmc_calib JSON line> [--out F]

For each kernel: the counters (KB -> bytes), the known read / write bytes, and
their ratios.  The ratio for 'k_rec_read' (128-B records, one lane per host,
8 x 16 B) is the read correction bench.py's roofline traffic applies to the
round kernel's FETCH_SIZE (MI355X_MICROARCH.md: calibrate the access width
before trusting an absolute)."""
import argparse
import csv
import glob
import json
import os


def counters(d, name):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == name:
                    k = r["Kernel_Name"].split("(")[0].split()[-1]
                    out[k] = out.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("known")
    ap.add_argument("--out")
    a = ap.parse_args()
    known = json.loads([l for l in open(a.known).read().splitlines() if l.startswith("{")][-1])
    fe, wr = counters(a.fetch_dir, "FETCH_SIZE"), counters(a.write_dir, "WRITE_SIZE")
    res = {}
    for k, kb in known.items():
        f, w = fe.get(k), wr.get(k)
        res[k] = {"known_read": kb["read"], "known_write": kb["write"], "fetch_size_bytes": f, "write_size_bytes": w,
                  "fetch_over_known": round(f / kb["read"], 4) if f is not None and kb["read"] else None,
                  "write_over_known": round(w / kb["write"], 4) if w is not None and kb["write"] else None}
    out = {"note": "FETCH_SIZE / WRITE_SIZE (rocprofv3, KB) per kernel against the bytes the kernel must move; "
                   "read correction = known / FETCH_SIZE of k_rec_read (the round kernel's record pattern)",
           "kernels": res}
    r = res.get("k_rec_read", {}).get("fetch_over_known")
    out["read_correction"] = round(1.0 / r, 4) if r else None
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
