#!/bin/bash
# round 4: phase stamps and loop iterations of k_round_ps (C3) and k_round_sp (C5 shard),
# then the C5 125 k-host shard as one engine and as a one-rank fused group
set -o pipefail
O=gpurun_out/r04_c5t
mkdir -p $O
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/ps_timing.py > $O/timing_c3.txt 2>&1 || { tail -5 $O/timing_c3.txt; exit 3; }
cat $O/timing_c3.txt
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 300 python3 scripts/ps_timing.py --workload c5 --hosts 125000 > $O/timing_c5.txt 2>&1 || { tail -5 $O/timing_c5.txt; exit 4; }
cat $O/timing_c5.txt
HOSTS_OUT=$O bash -c '
run() {
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" > $HOSTS_OUT/$n.json 2> $HOSTS_OUT/$n.err || { tail $HOSTS_OUT/$n.err; return 1; }
  python3 -c "
import json
d=json.loads(open(\"$HOSTS_OUT/$n.json\").read().strip().splitlines()[-1]); r=d[\"roofline\"]
print(\"$n\", round(d[\"value\"]/1e6,2), \"M\", r[\"kernel\"], r[\"avg_round_us\"], \"us/round\", r[\"packet_events_per_launch\"], \"pkt/round\")"
}
run c5_125k --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 &&
run c5_125k_group --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --group --exchange p2p'
