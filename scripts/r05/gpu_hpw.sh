#!/bin/bash
# round 5: hosts per wave in the persistent round (SHD_HPW) on the C3 headline, alternated
set -o pipefail
O=gpurun_out/r05_hpw
mkdir -p $O
for rep in 1 2; do
  for h in 64 32 48; do
    SHD_HPW=$h timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-reference-cpu --steps 4 --warmup 2 \
        > $O/hpw${h}_$rep.json 2> $O/hpw${h}_$rep.err || { tail -3 $O/hpw${h}_$rep.err; exit 2; }
    python3 -c "
import json; d=json.load(open('$O/hpw${h}_$rep.json')); r=d['roofline']
print('hpw $h rep $rep', round(d['value']/1e6,2), 'M', r['kernel'], r.get('avg_round_us'))"
  done
done
