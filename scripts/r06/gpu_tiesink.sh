#!/bin/bash
# round 6: k_sssp_tie_g with a heap level read in one LDS round trip (both children together) and no register
# resets in the preload (123 ms before), against k_sssp_tie_lds<true> (SHD_PC_TIE_KIND=st): parity, 10 k whole-ms build
set -o pipefail
O=gpurun_out/r06_tiesink
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests_g.log 2>&1 || exit 2
SHD_PC_TIE_HV8=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_g_hv8.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_g_$rep.log 2>&1 || exit 3
  echo "g_$rep $(tail -n 1 $O/apsp_g_$rep.log)" >> $O/summary.txt
  SHD_PC_TIE_KIND=st timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_st_$rep.log 2>&1 || exit 3
  echo "st_$rep $(tail -n 1 $O/apsp_st_$rep.log)" >> $O/summary.txt
done
