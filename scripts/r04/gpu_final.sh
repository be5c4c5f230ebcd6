#!/bin/bash
# round 4, last call: the whole GPU suite and smoke() on the final tree, then the
# TCP bench line with its CPU sample (the oracle on the box's cores)
set -o pipefail
O=gpurun_out/r04_final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "suite rc=$rc"
grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --workload tcp --steps 1 --warmup 0 > $O/tcp_bench.json 2> $O/tcp_bench.err || { tail -5 $O/tcp_bench.err; exit 3; }
tail -1 $O/tcp_bench.json
