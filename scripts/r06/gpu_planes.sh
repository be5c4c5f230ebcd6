#!/bin/bash
# round 6: the round shares in three planes (coalesced polls) against 48-B records (SHD_PS_AOS):
# parity of the persistent kernels, then C3 headline and the C5 shard, two alternations
set -o pipefail
O=gpurun_out/r06_planes
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_pathcache_gpu.py > $O/tests.log 2>&1 || exit 2
timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp.log 2>&1 || exit 2
run() {
  local tag=$1 lib=$2; shift 2
  SHDGPU_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" \
      > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])" >> $O/summary.txt
}
for rep in 1 2; do
  run c3_planes_$rep shadow-1_amd/libshdgpu.so --steps 4 --warmup 2
  run c3_aos_$rep shadow-1_amd/libshdgpu_aos.so --steps 4 --warmup 2
  run c5_planes_$rep shadow-1_amd/libshdgpu.so --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
  run c5_aos_$rep shadow-1_amd/libshdgpu_aos.so --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
done
