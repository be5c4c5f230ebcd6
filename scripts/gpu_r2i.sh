#!/bin/bash
# GPU suite, the headline bench, the hosts-per-GPU runs and the one-rank fused group
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_r2h.sh || exit 1
bash scripts/gpu_scale_hosts.sh || exit 2
timeout -k 10 300 python3 bench.py --group --exchange p2p --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 \
    > gpurun_out/gfused.json 2> gpurun_out/gfused.err || { tail gpurun_out/gfused.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/gfused.json')); print('group fused', d['value'], d['ms_per_step'])"
