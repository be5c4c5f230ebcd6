#!/bin/bash
# round 5: the queued frontier (default) against the half-wave pairs
# (SHD_PC_BF_PAIRS), with and without the LDS offsets (SHD_PC_NO_LDS_OFF)
set -o pipefail
O=gpurun_out/r05_bfq
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  SHD_PC_BF_PAIRS=1 timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/pairs_$rep.log 2>&1 || exit 3
  timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/queue_$rep.log 2>&1 || exit 4
  SHD_PC_NO_LDS_OFF=1 timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/queue_glboff_$rep.log 2>&1 || exit 5
  for k in pairs queue queue_glboff; do echo "rep $rep $k: $(tail -1 $O/${k}_$rep.log)"; done
done
