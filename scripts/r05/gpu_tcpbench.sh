#!/bin/bash
# the TCP leg after both transports / groups landed: one GPU at the usual size (65 536 hosts, twice), then
# the sharded group rehearsed with 2 ranks on the one GPU (host-memory transport) beside one engine at the
# same per-GPU size
set -o pipefail
mkdir -p gpurun_out/r05_tcpbench
timeout -k 10 600 python -u bench.py --workload tcp --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05_tcpbench/tcp_1gpu_a.json 2> gpurun_out/r05_tcpbench/tcp_1gpu_a.err && \
timeout -k 10 600 python -u bench.py --workload tcp --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05_tcpbench/tcp_1gpu_b.json 2> gpurun_out/r05_tcpbench/tcp_1gpu_b.err && \
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --workload tcp --comm host --hosts-per-gpu 8192 --steps 2 --warmup 1 \
    > gpurun_out/r05_tcpbench/tcp_2rank_rehearsal.json 2> gpurun_out/r05_tcpbench/tcp_2rank_rehearsal.err && \
timeout -k 10 600 python -u bench.py --workload tcp --hosts-per-gpu 16384 --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05_tcpbench/tcp_1gpu_16384.json 2> gpurun_out/r05_tcpbench/tcp_1gpu_16384.err
