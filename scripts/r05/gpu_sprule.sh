#!/bin/bash
# the sparse/dense rule on packet events per host-round and activity: C5's shard (one engine and
# the one-rank group), 250 k hosts, C4, C3 at 100 k hosts, two alternations
set -o pipefail
O=gpurun_out/r05_sprule
mkdir -p $O
run() {  # tag workload extra
  local tag=$1 wl=$2; shift 2
  timeout -k 10 400 python3 bench.py --workload $wl --steps 2 --warmup 2 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['batches'], r['avg_launch_us'])"
}
for rep in 1 2; do
  run c5_$rep c5 --hosts-per-gpu 125000
  run c5grp_$rep c5 --hosts-per-gpu 125000 --group
  run c5h250_$rep c5 --hosts-per-gpu 250000
  run c4_$rep c4
  run c3h100_$rep c3 --hosts-per-gpu 100000
done
