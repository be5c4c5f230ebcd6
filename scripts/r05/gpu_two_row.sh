#!/bin/bash
# round 5: two rows per workgroup (k_sssp_rows2_lds) against one (SHD_PC_ONE_ROW)
set -o pipefail
O=gpurun_out/r05_tworow
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    tests/test_pc_touches_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  SHD_PC_ONE_ROW=1 timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/one_$rep.log 2>&1 || exit 3
  timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/two_$rep.log 2>&1 || exit 4
  for k in one two; do echo "rep $rep $k: $(tail -1 $O/${k}_$rep.log)"; done
done
