#!/bin/bash
# the engine-group path at one rank (RCCL communicator): bench line + kernel-trace stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gp/trace -o run -- \
    python3 bench.py --group --steps 2 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 > gpurun_out/gp/bench.json 2> gpurun_out/gp/bench.err || { tail gpurun_out/gp/bench.err; exit 1; }
f=$(find gpurun_out/gp/trace -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/gp/group_kernel_stats.csv
find gpurun_out/gp/trace -name "*kernel_trace.csv" -delete
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/gp/group_kernel_stats.csv")))
for r in rows[:10]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>7s} avg {float(r['AverageNs'])/1e3:8.2f} us  {r['Percentage']}%")
PY
python3 -c "import json; d=json.load(open('gpurun_out/gp/bench.json')); print(d['value'], d['ms_per_step'])"
