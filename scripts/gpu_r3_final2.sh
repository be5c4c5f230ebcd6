#!/bin/bash
# round 3 end: the whole GPU suite, smoke(), the default bench line and the TCP bench line
set -o pipefail
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 3; }
cat $O/bench.json
timeout -k 10 600 python3 bench.py --workload tcp --steps 2 --warmup 1 > $O/tcp_bench.json 2> $O/tcp_bench.err || { tail $O/tcp_bench.err; exit 4; }
cat $O/tcp_bench.json
