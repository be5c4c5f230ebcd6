#!/bin/bash
# the TCP path on a group of engines (several processes on the one GPU, host-memory transport)
set -o pipefail
mkdir -p gpurun_out/r05_tcpgroup
timeout -k 10 900 python -u -m pytest tests/test_tcp_group_gpu.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r05_tcpgroup/tests.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_tcp_gpu.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05_tcpgroup/tcp_single.log 2>&1
