#!/bin/bash
# A/B of the bench value: without and with an environment setting ($1=VAR=value)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
for k in 0 1 2; do
  for v in A B; do
    if [ $v = B ]; then ENVV="$1"; else ENVV="SHD_AB_NONE=1"; fi
    env $ENVV timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/ab_$v$k.json 2> gpurun_out/ab_$v$k.err || { tail -5 gpurun_out/ab_$v$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v$k.json')); print('$v', round(d['value']/1e6,2), d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
