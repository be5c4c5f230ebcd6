#!/bin/bash
# round 6: k_round_sp with its hosts' records resident in LDS for the batch against records
# in HBM (SHD_SP_NO_LREC): parity of the sparse paths, then the C5 shard, two alternations
set -o pipefail
O=gpurun_out/r06_lrec
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_xgroup_procs_gpu.py > $O/tests.log 2>&1 || exit 2
run() {
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" \
      > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])" >> $O/summary.txt
}
SHD_SP_VERBOSE=1 run c5_lrec_0 --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 1
for rep in 1 2; do
  run c5_lrec_$rep --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
  SHD_SP_NO_LREC=1 run c5_hbm_$rep --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
done
