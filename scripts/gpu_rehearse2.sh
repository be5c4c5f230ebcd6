#!/bin/bash
# 3 ranks on one GPU: fused at 3 k hosts per rank, unfused at 10 k (is the 10 k fused timeout co-residency?)
set -o pipefail
mkdir -p gpurun_out/reh
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 3 --steps 3 --warmup 2 --no-cpu-baseline --comm host --hosts-per-gpu 3000 \
    > gpurun_out/reh/n3_3k.json 2> gpurun_out/reh/n3_3k.err || { tail -20 gpurun_out/reh/n3_3k.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/reh/n3_3k.json')); print('3x3k fused', d['value'], d['ms_per_step'], d['config']['exchange'])"
SHD_X_UNFUSED=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
    --master-port 29542 bench.py --gpus 3 --steps 3 --warmup 2 --no-cpu-baseline --comm host \
    > gpurun_out/reh/n3_unf.json 2> gpurun_out/reh/n3_unf.err || { tail -20 gpurun_out/reh/n3_unf.err; exit 2; }
python3 -c "import json; d=json.load(open('gpurun_out/reh/n3_unf.json')); print('3x10k unfused', d['value'], d['ms_per_step'], d['config']['exchange'])"
