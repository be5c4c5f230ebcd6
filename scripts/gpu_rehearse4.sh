#!/bin/bash
# the bench's N > 1 path with 4 ranks on one GPU, small enough (4 x 4000 hosts = 252 blocks) to run fused
set -o pipefail
mkdir -p gpurun_out/reh
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29574 bench.py --gpus 4 --steps 3 --warmup 2 --no-cpu-baseline --comm host --hosts-per-gpu 4000 \
    > gpurun_out/reh/n4.json 2> gpurun_out/reh/n4.err || { tail -20 gpurun_out/reh/n4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/reh/n4.json')); print(4, d['value'], d['ms_per_step'], d['rounds'], d['config']['exchange'], d['apsp']['sharded_build_ms'], d['first_touch'])"
