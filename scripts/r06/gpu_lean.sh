#!/bin/bash
# round 6: (1) tied rows, k_sssp_tie_lds with the next pop's arcs preloaded: parity + 10 k build times;
# (2) the lean instantiations of k_round_tl / _ps / _sp (models with feat == 0): parity (engine,
# full-size fixtures), then A/B against the general ones (libshdgpu_nolean.so) on C3 (10 k, 100 k),
# C4 and the C5 shard, two alternations
set -o pipefail
O=gpurun_out/r06_lean
mkdir -p $O
T="timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
$T tests/test_pathcache_gpu.py > $O/tests_pc.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp.log 2>&1 && \
$T tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_model_gpu.py > $O/tests_eng.log 2>&1 || exit 2
run() {
  local tag=$1 lib=$2; shift 2
  SHDGPU_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])" >> $O/summary.txt
}
for rep in 1 2; do
  for v in lean nolean; do
    L=shadow-1_amd/libshdgpu.so; [ $v = nolean ] && L=shadow-1_amd/libshdgpu_nolean.so
    run c3_${v}_$rep $L --steps 4 --warmup 2
    [ $rep = 1 ] || continue
    run c3h100_${v}_$rep $L --hosts-per-gpu 100000 --steps 2 --warmup 2
    run c4_${v}_$rep $L --workload c4 --steps 2 --warmup 2
    run c5_${v}_$rep $L --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
  done
done
