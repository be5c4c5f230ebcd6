#!/bin/bash
# BASELINE C5 on one GPU: 1M hosts (the whole model) on a geometric topology
set -o pipefail
mkdir -p gpurun_out
for cfg in "1000000 10000" "1000000 50000"; do
  set -- $cfg
  echo "hosts=$1 vertices=$2"
  timeout -k 10 500 python -u bench.py --hosts-per-gpu $1 --vertices $2 --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline \
      > gpurun_out/c5_$1_$2.json 2> gpurun_out/c5_$1_$2.err || { tail -20 gpurun_out/c5_$1_$2.err; exit 1; }
  cat gpurun_out/c5_$1_$2.json; grep -v amdgpu.ids gpurun_out/c5_$1_$2.err
done
