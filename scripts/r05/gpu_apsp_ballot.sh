#!/bin/bash
# the two-row kernel walking only its non-empty bit words (ballot + readlane, the default) against every
# chunk's four shuffles (SHD_SSSP_BALLOT=0): the path-cache suites first, then the 10 k table, alternating
set -o pipefail
O=gpurun_out/r05_apsp_ballot
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    tests/test_pc_touches_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  SHDGPU_LIB=shadow-1_amd/libshdgpu_pcv_noballot.so timeout -k 10 200 python -u scripts/r05/apsp_once.py > $O/shfl_$rep.log 2>&1 || exit 3
  timeout -k 10 200 python -u scripts/r05/apsp_once.py > $O/ballot_$rep.log 2>&1 || exit 4
  echo "rep $rep shfl: $(tail -1 $O/shfl_$rep.log)  ballot: $(tail -1 $O/ballot_$rep.log)"
done
