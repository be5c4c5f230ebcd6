#!/bin/bash
# A/B of the per-host LDS capacities (default 6/5 against 8/8, libshdgpu_var.so): one-rank fused group and the headline.
# (Built while engine.hip read kDueCap / kSendCap from SHD_DUE_CAP / SHD_SEND_CAP: make variant VARIANT_FLAGS="-DSHD_DUE_CAP=8 -DSHD_SEND_CAP=8";
# the product keeps plain constants.)
set -o pipefail
mkdir -p gpurun_out/ab
G="--group --exchange p2p --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
H="--steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
for rep in 1 2; do
for v in def var; do
  if [ $v = var ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_var.so; else unset SHDGPU_LIB; fi
  timeout -k 10 200 python3 bench.py $G > gpurun_out/ab/g_$v.json 2> gpurun_out/ab/g_$v.err || { tail gpurun_out/ab/g_$v.err; exit 1; }
  timeout -k 10 200 python3 bench.py $H > gpurun_out/ab/h_$v.json 2> gpurun_out/ab/h_$v.err || { tail gpurun_out/ab/h_$v.err; exit 2; }
  python3 -c "import json; g=json.load(open('gpurun_out/ab/g_$v.json')); h=json.load(open('gpurun_out/ab/h_$v.json')); print('$rep $v group', round(g['value']/1e6,1), 'single', round(h['value']/1e6,1))"
done
done
