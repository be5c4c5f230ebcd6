#!/bin/bash
# C4 (56.5 k hosts, ~14 % active per round) under the new sparse defaults: the default, the old
# 8 % switch, and smaller sparse blocks (SHD_SP_HOSTS 128 / 192 / 256, sparse throughout)
set -o pipefail
O=gpurun_out/r05_spc4
mkdir -p $O
run() {  # tag (env in front) extra
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py --workload c4 --steps 2 --warmup 2 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['batches'], r['avg_launch_us'])"
}
for rep in 1 2; do
  run c4_def_$rep
  SHD_SP_DENSE_FRAC=0.08 run c4_f08_$rep
  SHD_SP_HOSTS=128 run c4_s128_$rep
  SHD_SP_HOSTS=192 run c4_s192_$rep
  SHD_SP_HOSTS=256 run c4_s256_$rep
done
