#!/bin/bash
# round 4: the whole GPU suite (no -x: every failure listed), then smoke()
set -o pipefail
O=gpurun_out/r04_suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "suite rc=$?"
grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -30
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $O/smoke.log
