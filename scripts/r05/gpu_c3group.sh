#!/bin/bash
# round 5: the C3 headline through the one-rank group (the path every rank of
# an N > 1 run takes) against the single engine
set -o pipefail
O=gpurun_out/r05_c3group
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --group --no-cpu-baseline --no-reference-cpu --steps 4 --warmup 2 \
      > $O/group_$rep.json 2> $O/group_$rep.err || { tail -5 $O/group_$rep.err; exit 2; }
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-reference-cpu --steps 4 --warmup 2 \
      > $O/single_$rep.json 2> $O/single_$rep.err || { tail -5 $O/single_$rep.err; exit 3; }
  for k in group single; do python3 -c "
import json; d=json.load(open('$O/${k}_$rep.json')); r=d['roofline']
print('$k rep $rep', round(d['value']/1e6,2), 'M', r['kernel'], r.get('avg_round_us'), d['config'].get('exchange', ''))"; done
done
