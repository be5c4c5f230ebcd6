#!/bin/bash
# A/B of the bench value: the default library against libshdgpu_var.so
# (make -C shadow-1_amd variant VARIANT_FLAGS=...), alternating A B A B A B
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
for k in 0 1 2; do
  for v in A B; do
    if [ $v = B ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_var.so; else unset SHDGPU_LIB; fi
    timeout -k 10 150 python bench.py --no-cpu-baseline --lossy-edge-loss-max 0 $AB_ARGS > gpurun_out/ab_$v$k.json 2> gpurun_out/ab_$v$k.err || { tail -5 gpurun_out/ab_$v$k.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v$k.json')); print('$v', round(d['value']/1e6,2), d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
