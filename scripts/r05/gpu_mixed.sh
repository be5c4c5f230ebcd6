#!/bin/bash
# both transports in one TCP-path model: the mixed_* reference fixtures, and the echo cases (no regression)
set -o pipefail
mkdir -p gpurun_out/r05_mixed
timeout -k 10 600 python -u -m pytest tests/test_tcp_gpu.py -x -v --timeout 300 --timeout-method thread \
    -k "mixed or ref_epoll or loopback or shared_hosts or scaled" > gpurun_out/r05_mixed/tests.log 2>&1
