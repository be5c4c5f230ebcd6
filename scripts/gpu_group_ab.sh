#!/bin/bash
# the engine-group path at one rank: peer-to-peer transport vs RCCL all-to-all
set -o pipefail
mkdir -p gpurun_out
for x in p2p rccl; do
  timeout -k 10 300 python3 bench.py --group --exchange $x --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 \
      > gpurun_out/group_$x.json 2> gpurun_out/group_$x.err || { tail gpurun_out/group_$x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/group_$x.json')); print('$x', d['value'], d['ms_per_step'], d['config']['exchange'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])"
done
