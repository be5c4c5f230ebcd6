#!/bin/bash
# round 6: the path-cache GPU suite (tied graphs at half-millisecond latencies added)
set -o pipefail
O=gpurun_out/r06_pctests
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests.log 2>&1
