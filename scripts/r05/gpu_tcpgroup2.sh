#!/bin/bash
# the TCP group after its control all-gathers moved to kept device buffers: the group suite (with the
# one-rank RCCL run) and the two-rank rehearsal of the bench leg
set -o pipefail
mkdir -p gpurun_out/r05_tcpgroup2
timeout -k 10 900 python -u -m pytest tests/test_tcp_group_gpu.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r05_tcpgroup2/tests.log 2>&1 && \
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --workload tcp --comm host --hosts-per-gpu 8192 --steps 2 --warmup 1 \
    > gpurun_out/r05_tcpgroup2/tcp_2rank_rehearsal.json 2> gpurun_out/r05_tcpgroup2/tcp_2rank_rehearsal.err
