#!/bin/bash
# round 6: a predicted all-tied build with its ties counted by two streaming passes (least exact predecessor
# distance, then the count at it) instead of an in-arc walk: parity, the 10 k build, against SHD_PC_NO_TIE_PREDICT
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tiecnt
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py tests/test_pc_touches_gpu.py > $O/tests.log 2>&1 || exit 2
SHD_PC_TIE_HV8=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_hv8.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_pred_$rep.log 2>&1 || exit 3
  echo "pred_$rep $(tail -n 1 $O/apsp_pred_$rep.log)" >> $O/summary.txt
  SHD_PC_NO_TIE_PREDICT=1 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_full_$rep.log 2>&1 || exit 3
  echo "full_$rep $(tail -n 1 $O/apsp_full_$rep.log)" >> $O/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 scripts/r06/tie_once.py > $O/tr.log 2>&1 || exit 4
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv && rm -rf $O/tr
