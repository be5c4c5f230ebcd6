#!/bin/bash
# sparse against dense batches on one engine: the default switch (8 % active hosts per round),
# higher thresholds (SHD_SP_DENSE_FRAC) and the sparse kernel throughout (SHD_SP_HOSTS), at the
# C5 shard (125 k hosts) and 250 k hosts; batch counts per run from bench's roofline
set -o pipefail
O=gpurun_out/r05_spdense
mkdir -p $O
run() {  # tag hosts (env in front)
  local tag=$1 hosts=$2
  timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu $hosts --steps 2 --warmup 2 \
      --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['batches'], r['avg_launch_us'])"
}
for rep in 1 2; do
  run h125_def_$rep 125000
  SHD_SP_HOSTS=256 run h125_force256_$rep 125000
  SHD_SP_DENSE_FRAC=0.16 run h125_f16_$rep 125000
  SHD_SP_DENSE_FRAC=0.3 run h125_f30_$rep 125000
  run h250_def_$rep 250000
  SHD_SP_HOSTS=512 run h250_force512_$rep 250000
  SHD_SP_DENSE_FRAC=0.16 run h250_f16_$rep 250000
  SHD_SP_DENSE_FRAC=0.3 run h250_f30_$rep 250000
done
