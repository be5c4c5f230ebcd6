#!/bin/bash
# C3 at 100 k hosts (k_round_tl): 45.6 µs a round this round against 43.1 in round 3 -- with the
# ambiguous-round restore point off (SHD_NO_REPLAY) against the default, two alternations
set -o pipefail
O=gpurun_out/r05_tlreg
mkdir -p $O
run() {
  local tag=$1
  timeout -k 10 400 python3 bench.py --workload c3 --hosts-per-gpu 100000 --steps 2 --warmup 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['avg_in_kernel_us'])"
}
for rep in 1 2; do
  run def_$rep
  SHD_NO_REPLAY=1 run norep_$rep
done
