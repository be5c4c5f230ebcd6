#!/bin/bash
# hosts per block of the sparse persistent round (SHD_SP_HOSTS) at the C5 shard (125 k hosts; default 512:
# 245 blocks, one per CU) against 256 / 384 (489 / 326 blocks, up to two per CU), two alternations
set -o pipefail
O=gpurun_out/r05_sph
mkdir -p $O
for rep in 1 2; do
  for sph in 512 256 384; do
    SHD_SP_HOSTS=$sph timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 \
        --no-cpu-baseline > $O/sph${sph}_$rep.json 2> $O/sph${sph}_$rep.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/sph${sph}_$rep.json').read().strip().splitlines()[-1]); print('rep $rep sph $sph', d['value'], d['ms_per_step'])"
  done
done
