#!/bin/bash
# round 5: the TCP GPU tests (mailbox overflow), then the default bench line
set -o pipefail
O=gpurun_out/r05_tb
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_tcp_gpu.py > $O/tcp_tests.log 2>&1; rc=$?
echo "tcp tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tcp_tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -5 $O/bench.err; cat $O/bench.json
