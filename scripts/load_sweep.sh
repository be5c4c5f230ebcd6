#!/bin/bash
# per-round cost against the offered load (messages in flight per host):
# the intercept is the round's fixed cost, the slope the per-event cost
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/load_sweep.log
for ld in 1 4 16 64; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --load $ld --steps 4 > gpurun_out/ls_$ld.json 2> gpurun_out/ls_$ld.err || { tail -5 gpurun_out/ls_$ld.err; exit 1; }
  python - "$ld" >> gpurun_out/load_sweep.log <<'EOF'
import json, sys
ld = sys.argv[1]
d = json.load(open(f"gpurun_out/ls_{ld}.json"))
r = d["roofline"]
ev_round = d["all_events_per_s"] * d["ms_per_step"] / 1e3 / (d["rounds"] / (d["steps"] + d["warmup"]))
print(f"load {ld:>3}: {d['value'] / 1e6:7.2f} M pkt ev/s  launch {r['avg_launch_us']:6.2f} us  in-kernel "
      f"{r['avg_in_kernel_us']:6.2f} us  events/round {ev_round:8.0f}")
EOF
done
cat gpurun_out/load_sweep.log
