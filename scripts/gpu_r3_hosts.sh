#!/bin/bash
# round 3: per-GPU shard of the north star (C5 model, 125 k hosts) as one engine and as a
# one-rank fused group; C4 (Tor-scale, 56.5 k hosts); C3 at 100 k hosts
set -o pipefail
O=${HOSTS_OUT:-gpurun_out/r03/hosts}
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python3 -c "
import json
d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$n', round(d['value']/1e6,2), 'M', r['kernel'], r['avg_round_us'], 'us/round', r['packet_events_per_launch'], 'pkt/round', d['config'].get('exchange'))"
}
run c5_125k --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 &&
run c5_125k_group --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --group --exchange p2p &&
run c3_group --group --exchange p2p --steps 4 --warmup 2 &&
run c4 --workload c4 --steps 2 --warmup 2 &&
run c3_100k --hosts-per-gpu 100000 --steps 2 --warmup 2
