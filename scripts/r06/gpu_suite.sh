#!/bin/bash
# round 6: the whole GPU suite, then the driver's default bench line (C3 headline)
set -o pipefail
O=gpurun_out/r06_suite
mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -x -q -m gpu --timeout 900 --timeout-method thread \
    > $O/tests.log 2>&1; echo "pytest rc=$?" >> $O/tests.log
tail -3 $O/tests.log
grep -q "pytest rc=0" $O/tests.log && \
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
