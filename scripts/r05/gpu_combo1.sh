#!/bin/bash
# round 5: path cache (relabelled, flattened frontier) + TCP (device first touch)
# tests, the APSP A/B, the TCP bench line
set -o pipefail
O=gpurun_out/r05_combo1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    tests/test_tcp_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r05/gpu_apsp_ab.sh > $O/apsp_ab.out 2>&1; echo "apsp ab rc=$?"; grep -v "^tests/" $O/apsp_ab.out | tail -40
timeout -k 10 300 python -u scripts/r05/tcp_wide_probe.py > $O/wide.log 2>&1; echo "probe rc=$?"; cat $O/wide.log
timeout -k 10 900 python -u bench.py --workload tcp --steps 3 --warmup 1 > $O/tcp_bench.json 2> $O/tcp_bench.err
echo "tcp bench rc=$?"; tail -3 $O/tcp_bench.err; cat $O/tcp_bench.json
