#!/bin/bash
# round 5: the last call on the final tree -- the whole -m gpu suite, smoke(),
# then the C3 headline refresh (bench line, rocprof timed region, PMC traffic,
# SQ counters) for the final engine source
set -o pipefail
O=gpurun_out/${FINAL_OUT:-r05_final}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.log
