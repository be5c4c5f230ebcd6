#!/bin/bash
# Packet events/s against hosts per GPU (one GPU): the per-round fixed cost
# amortised over more hosts.  Outputs gpurun_out/scale_<H>_<V>.json
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-"100000 10000" "125000 50000" "1000000 50000"}; do
  set -- $cfg
  echo "hosts=$1 vertices=$2"
  timeout -k 10 ${TL:-240} python -u bench.py --hosts-per-gpu $1 --vertices $2 --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline \
      > gpurun_out/scale_$1_$2.json 2> gpurun_out/scale_$1_$2.err || { tail -20 gpurun_out/scale_$1_$2.err; exit 1; }
  cat gpurun_out/scale_$1_$2.json
done
