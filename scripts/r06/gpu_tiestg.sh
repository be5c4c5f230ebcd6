#!/bin/bash
# round 6: the LDS tie kernel with the vertex states in global scratch (heap-only LDS, 16 rows per CU)
# against states in LDS (SHD_PC_TIE_STG=0): tie parity both ways, then the 10 k whole-ms build, two alternations
set -o pipefail
O=gpurun_out/r06_tiestg
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests_stg.log 2>&1 || exit 2
SHD_PC_TIE_STG=0 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_lds.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_stg_$rep.log 2>&1 || exit 3
  echo "stg_$rep $(tail -n 1 $O/apsp_stg_$rep.log)" >> $O/summary.txt
  SHD_PC_TIE_STG=0 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_lds_$rep.log 2>&1 || exit 3
  echo "lds_$rep $(tail -n 1 $O/apsp_lds_$rep.log)" >> $O/summary.txt
done
