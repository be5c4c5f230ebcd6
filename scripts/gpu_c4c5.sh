#!/bin/bash
# BASELINE C4 on one GPU, and C5 (1 M hosts) split over 2 ranks sharing one GPU (rehearsal of its N > 1 path)
set -o pipefail
mkdir -p gpurun_out/hosts
timeout -k 10 300 python3 bench.py --workload c4 --steps 2 --warmup 2 --no-cpu-baseline \
    > gpurun_out/hosts/c4_1gpu.json 2> gpurun_out/hosts/c4_1gpu.err || { tail gpurun_out/hosts/c4_1gpu.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/hosts/c4_1gpu.json')); r=d['roofline']; print('c4', d['config']['hosts'], round(d['value']/1e6,1), d['ms_per_step'], d['rounds'], r['avg_launch_us'])"
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29561 bench.py --gpus 2 --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --comm host \
    > gpurun_out/hosts/c5_reh2.json 2> gpurun_out/hosts/c5_reh2.err || { tail -20 gpurun_out/hosts/c5_reh2.err; exit 2; }
python3 -c "import json; d=json.load(open('gpurun_out/hosts/c5_reh2.json')); print('c5 rehearsal x2', d['config']['hosts'], round(d['value']/1e6,1), d['ms_per_step'], d['rounds'], d['config']['exchange'], d['first_touch'])"
