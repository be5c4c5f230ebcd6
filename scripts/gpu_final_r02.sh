#!/bin/bash
# round-end check: the whole GPU suite and smoke(), as the driver runs them
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/final_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/final_tests.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail gpurun_out/final_smoke.log; exit 2; }
tail -2 gpurun_out/final_smoke.log
