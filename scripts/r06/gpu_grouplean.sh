#!/bin/bash
# round 6: the lean fused group kernels (k_round_px / k_round_spx, feat == 0): the group parity tests,
# then the one-rank group A/B (lean against libshdgpu_nolean.so) at C3 10 k and the C5 shard
set -o pipefail
O=gpurun_out/r06_grouplean
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_xgroup_procs_gpu.py tests/test_fullsize_gpu.py -k "group or sharded or parts" > $O/tests.log 2>&1 || exit 2
run() {
  local tag=$1 lib=$2; shift 2
  SHDGPU_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 --group "$@" \
      > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])" >> $O/summary.txt
}
for rep in 1 2; do
  run c3g_lean_$rep shadow-1_amd/libshdgpu.so --steps 4 --warmup 2
  run c3g_nolean_$rep shadow-1_amd/libshdgpu_nolean.so --steps 4 --warmup 2
  run c5g_lean_$rep shadow-1_amd/libshdgpu.so --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
  run c5g_nolean_$rep shadow-1_amd/libshdgpu_nolean.so --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
done
