#!/bin/bash
# round 4: the TCP path's tracker [node] lines against the reference loop, the path cache's
# one-cache protocol, the co-simulation tests
set -o pipefail
O=gpurun_out/r04_tcpnode
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_tcp_gpu.py tests/test_pc_touches_gpu.py tests/test_ingress_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "rc=$?"
grep -E "PASSED|FAILED|^E " $O/tests.log | tail -40
