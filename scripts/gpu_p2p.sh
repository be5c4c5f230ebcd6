#!/bin/bash
# the multi-process group tests (all-to-all and peer-to-peer transports)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_xgroup_procs_gpu.py > gpurun_out/tp2p.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tp2p.log | tail -15
exit $rc
