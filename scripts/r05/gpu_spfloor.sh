#!/bin/bash
# the sparse block's floor of 256 hosts on engines between ~33 k and 131 k hosts: the C5 model at
# 50 k hosts (196 blocks of 256, under one per CU) against blocks of 128 (391), sparse throughout
# both ways, and the default; two alternations
set -o pipefail
O=gpurun_out/r05_spfloor
mkdir -p $O
run() {
  local tag=$1
  timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu 50000 --steps 2 --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['batches'], r['avg_launch_us'])"
}
for rep in 1 2; do
  run def_$rep
  SHD_SP_HOSTS=256 run s256_$rep
  SHD_SP_HOSTS=128 run s128_$rep
done
