#!/bin/bash
# the one-rank engine group at the C5 shard: the sparse fused round's hosts per block and the
# sparse/dense switch (default now: about two blocks per CU, switch at 30 % active hosts)
set -o pipefail
O=gpurun_out/r05_spgroup
mkdir -p $O
run() {  # tag hosts (env in front) extra
  local tag=$1 hosts=$2; shift 2
  timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu $hosts --steps 2 --warmup 2 \
      --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['batches'], r['avg_launch_us'])"
}
for rep in 1 2; do
  run single_def_$rep 125000
  run grp_def_$rep 125000 --group
  SHD_SP_HOSTS=256 run grp_force256_$rep 125000 --group
  SHD_SP_HOSTS=512 run grp_force512_$rep 125000 --group
  SHD_SP_DENSE_FRAC=0.08 run grp_f08_$rep 125000 --group
done
