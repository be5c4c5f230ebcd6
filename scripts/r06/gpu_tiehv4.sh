#!/bin/bash
# round 6: the tie kernel's 4-B heap values on whole-number weights (6 B a heap entry, up to 26 rows per CU)
# against 8-B values (SHD_PC_TIE_HV8): tie parity both ways, then the 10 k whole-ms build, two alternations
set -o pipefail
O=gpurun_out/r06_tiehv4
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests_hv4.log 2>&1 || exit 2
SHD_PC_TIE_HV8=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_hv8.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_hv4_$rep.log 2>&1 || exit 3
  echo "hv4_$rep $(tail -n 1 $O/apsp_hv4_$rep.log)" >> $O/summary.txt
  SHD_PC_TIE_HV8=1 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_hv8_$rep.log 2>&1 || exit 3
  echo "hv8_$rep $(tail -n 1 $O/apsp_hv8_$rep.log)" >> $O/summary.txt
done
