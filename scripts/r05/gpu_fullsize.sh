#!/bin/bash
# round 5: the full-size tests in one process (the engines' state copies freed
# with them), and the path-cache tests with the two-row queue depth 2
set -o pipefail
O=gpurun_out/r05_fullsize
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_fullsize_gpu.py \
    tests/test_pathcache_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -20
