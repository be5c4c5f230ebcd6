#!/bin/bash
# round 6: k_round_sp's last-pass counter atomics after the round's share (default) against before its drain
# (libshdgpu_var.so, -DSHD_SP_CNT_EARLY): sparse parity, then the C5 shard, three alternations
set -o pipefail
O=gpurun_out/r06_cnt
rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_engine_gpu.py tests/test_fullsize_gpu.py > $O/tests.log 2>&1 || exit 2
run() {
  local tag=$1 lib=$2; shift 2
  SHDGPU_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" \
      > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])" >> $O/summary.txt
}
for rep in 1 2 3; do
  run c5_late_$rep shadow-1_amd/libshdgpu.so --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
  run c5_early_$rep shadow-1_amd/libshdgpu_var.so --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
done
