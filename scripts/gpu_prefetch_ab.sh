#!/bin/bash
# the group tests, then the one-rank fused group: headers prefetched with the batch summaries (default) against libshdgpu_old.so
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_xgroup_procs_gpu.py > gpurun_out/tfuse.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tfuse.log | tail -5
[ $rc -eq 0 ] || exit 1
G="--group --exchange p2p --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
for rep in 1 2; do
for v in new old; do
  if [ $v = old ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_old.so; else unset SHDGPU_LIB; fi
  timeout -k 10 200 python3 bench.py $G > gpurun_out/ab/p_$v.json 2> gpurun_out/ab/p_$v.err || { tail gpurun_out/ab/p_$v.err; exit 2; }
  python3 -c "import json; g=json.load(open('gpurun_out/ab/p_$v.json')); r=g['roofline']; print('$rep $v group', round(g['value']/1e6,1), g['ms_per_step'], r['avg_launch_us'])"
done
done
