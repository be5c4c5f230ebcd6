#!/bin/bash
# round 5: ambiguous unprotected rounds recovered by replay from the last restore point
set -o pipefail
O=gpurun_out/r05_replay
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_engine_gpu.py \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -30
