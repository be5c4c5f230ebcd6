#!/bin/bash
# round 5: path-cache tie rows (k_sssp_tie_parents) on the GPU: parity tests,
# then the APSP build time on a tie-free and an integer-latency 10 k graph
set -o pipefail
O=gpurun_out/r05_tie
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    tests/test_pc_touches_gpu.py tests/test_ingress_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/r05/apsp_ties.py > $O/apsp.log 2>&1; echo "apsp rc=$?"; cat $O/apsp.log
