#!/bin/bash
# after the socket-layout fix: the TCP suites (one engine, groups) and the TCP leg twice
set -o pipefail
mkdir -p gpurun_out/r05_tcpall
timeout -k 10 600 python -u -m pytest tests/test_tcp_gpu.py tests/test_tcp_group_gpu.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r05_tcpall/tests.log 2>&1 && \
timeout -k 10 600 python -u bench.py --workload tcp --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05_tcpall/tcp_1gpu_a.json 2> gpurun_out/r05_tcpall/tcp_1gpu_a.err && \
timeout -k 10 600 python -u bench.py --workload tcp --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05_tcpall/tcp_1gpu_b.json 2> gpurun_out/r05_tcpall/tcp_1gpu_b.err
