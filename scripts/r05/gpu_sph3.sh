#!/bin/bash
# the new sparse default (about two blocks per CU): C5 shard and 250 k hosts on one engine,
# and the one-rank group at the C5 shard (default against the old one block of 512 per CU)
set -o pipefail
O=gpurun_out/r05_sph3
mkdir -p $O
run() {  # tag hosts extra...
  local tag=$1 hosts=$2; shift 2
  timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu $hosts --steps 2 --warmup 2 \
      --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'])"
}
run h125_default 125000
run h250_default 250000
run grp_h125_default 125000 --group
SHD_SP_HOSTS=512 run grp_h125_s512 125000 --group
run grp_h125_default_2 125000 --group
