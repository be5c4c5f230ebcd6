#!/bin/bash
# round 5: batched path lookups (shd_pc_lookup_batch) -- path-cache + TCP tests,
# the wide-window probe, then the TCP bench line (wall-inclusive rate)
set -o pipefail
O=gpurun_out/r05_tcp2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
    tests/test_tcp_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/r05/tcp_wide_probe.py > $O/wide.log 2>&1; echo "probe rc=$?"; cat $O/wide.log
timeout -k 10 900 python -u bench.py --workload tcp --steps 3 --warmup 1 > $O/tcp_bench.json 2> $O/tcp_bench.err
echo "tcp bench rc=$?"; tail -3 $O/tcp_bench.err; cat $O/tcp_bench.json
