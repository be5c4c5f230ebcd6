#!/bin/bash
# round 6: the tie kernel's grid sized for as many rows per block against every slot filled (SHD_PC_TIE_FILL):
# tie parity, then the 10 k whole-ms build, two alternations
set -o pipefail
O=gpurun_out/r06_tiefill
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_bal_$rep.log 2>&1 || exit 3
  echo "bal_$rep $(tail -n 1 $O/apsp_bal_$rep.log)" >> $O/summary.txt
  SHD_PC_TIE_FILL=1 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_fill_$rep.log 2>&1 || exit 3
  echo "fill_$rep $(tail -n 1 $O/apsp_fill_$rep.log)" >> $O/summary.txt
done
