#!/bin/bash
# the TCP leg with both transports (a datagram process on every host beside the echo pairs), 16 384 hosts,
# beside the echo-only model at the same size
set -o pipefail
mkdir -p gpurun_out/r05_tcpmixed
timeout -k 10 900 python -u bench.py --workload tcp --tcp-udp --hosts-per-gpu 16384 --steps 2 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r05_tcpmixed/mixed_16384.json 2> gpurun_out/r05_tcpmixed/mixed_16384.err && \
timeout -k 10 600 python -u bench.py --workload tcp --hosts-per-gpu 16384 --steps 2 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r05_tcpmixed/echo_16384.json 2> gpurun_out/r05_tcpmixed/echo_16384.err
