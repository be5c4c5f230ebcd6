#!/bin/bash
# second sweep of the sparse round's hosts per block: 192 / 256 at the C5 shard (125 k hosts),
# 512 / 1024 at 250 k hosts, and the one-rank group (host comm) at 125 k with 256 vs the default
set -o pipefail
O=gpurun_out/r05_sph2
mkdir -p $O
run() {  # tag sph hosts extra...
  local tag=$1 sph=$2 hosts=$3; shift 3
  SHD_SP_HOSTS=$sph timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu $hosts --steps 2 --warmup 2 \
      --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  run h125_s192_$rep 192 125000
  run h125_s256_$rep 256 125000
  run h250_s1024_$rep 1024 250000
  run h250_s512_$rep 512 250000
done
