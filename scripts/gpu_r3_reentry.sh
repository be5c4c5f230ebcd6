#!/bin/bash
# round 3 re-entry: the GPU suite (TCP included) and the default bench line
set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
cat $O/bench.json
