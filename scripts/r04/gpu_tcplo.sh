#!/bin/bash
# round 4: loopback TCP (network_interface.c:548-555) and the round-robin qdisc on the GPU
# against the reference loop's fixtures, with the rest of the TCP tests
set -o pipefail
O=gpurun_out/r04_tcplo
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_tcp_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "rc=$?"
grep -E "PASSED|FAILED|^E " $O/tests.log | tail -40
