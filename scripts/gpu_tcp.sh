#!/bin/bash
# the TCP path on the GPU: its test against the reference fixtures
set -o pipefail
O=gpurun_out/tcp
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_tcp_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -30 $O/tests.log
exit $rc
