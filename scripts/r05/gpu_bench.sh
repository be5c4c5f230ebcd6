#!/bin/bash
# round 5: the default bench line (N = 1), with the reference's own CPU loop
set -o pipefail
O=gpurun_out/r05_bench${1:-}
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -5 $O/bench.err; cat $O/bench.json
