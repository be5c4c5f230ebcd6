#!/bin/bash
# round 3: k_round_sp hosts-per-block sweep on the C5 shard (125 k hosts)
set -o pipefail
O=gpurun_out/r03/sph
mkdir -p $O
for sph in 512 256 192 128; do
  SHD_SP_HOSTS=$sph timeout -k 10 300 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 > $O/c5_$sph.json 2> $O/c5_$sph.err || { tail $O/c5_$sph.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c5_$sph.json').read().strip().splitlines()[-1]); r=d['roofline']
print('sph $sph', round(d['value']/1e6,2), 'M', r['kernel'], r['avg_round_us'], 'us/round', r['active_hosts_per_launch'], 'active/round')"
done
