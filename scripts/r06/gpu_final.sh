#!/bin/bash
# round 6, final tree: the whole GPU suite, smoke(), then the driver's default bench line (C3 headline)
set -o pipefail
O=${O:-gpurun_out/r06_final}
rm -rf $O; mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread \
    > $O/tests.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/tests.log
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo final done
