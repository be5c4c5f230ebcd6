#!/bin/bash
# fused round LDS (kRxCap / kXDefCap 2, default) against libshdgpu_old.so (4 / 4): one-rank fused group at 100 k and 10 k hosts
set -o pipefail
mkdir -p gpurun_out/ab
for hosts in 100000 10000; do
for v in new old; do
  if [ $v = old ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_old.so; else unset SHDGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --group --exchange p2p --hosts-per-gpu $hosts --steps 2 --warmup 2 --no-cpu-baseline \
      --lossy-edge-loss-max 0 > gpurun_out/ab/px_$v.json 2> gpurun_out/ab/px_$v.err || { tail gpurun_out/ab/px_$v.err; exit 2; }
  python3 -c "import json; g=json.load(open('gpurun_out/ab/px_$v.json')); r=g['roofline']; print('$hosts $v', round(g['value']/1e6,1), g['ms_per_step'], r['avg_launch_us'])"
done
done
