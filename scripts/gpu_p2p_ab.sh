#!/bin/bash
# group tests (both transports) + one-rank group bench: fused fold+put vs split
set -o pipefail
mkdir -p gpurun_out
./scripts/gpu_p2p.sh || exit 1
for v in direct staged; do
  unset SHD_X_STAGED; [ $v = staged ] && export SHD_X_STAGED=1
  timeout -k 10 300 python3 bench.py --group --exchange p2p --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 \
      > gpurun_out/group_$v.json 2> gpurun_out/group_$v.err || { tail gpurun_out/group_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/group_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])"
done
