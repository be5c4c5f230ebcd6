#!/bin/bash
# round 6: the final tree's 10 k APSP builds (tie-free and all-tied), three repetitions
set -o pipefail
O=gpurun_out/r06_tiecheck
rm -rf $O; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_$rep.log 2>&1 || exit 3
  echo "final_$rep $(tail -n 1 $O/apsp_$rep.log)" >> $O/summary.txt
done
