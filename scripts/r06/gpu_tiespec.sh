#!/bin/bash
# round 6: k_sssp_tie_g with the next pop's arcs speculated from the heap top after the sink, against without
# (SHD_PC_TIE_NOSPEC): tie parity both ways (4-B and 8-B values), the 10 k whole-ms build, two alternations
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tiespec
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests.log 2>&1 || exit 2
SHD_PC_TIE_HV8=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_hv8.log 2>&1 || exit 2
SHD_PC_TIE_NOSPEC=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_nospec.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_spec_$rep.log 2>&1 || exit 3
  echo "spec_$rep $(tail -n 1 $O/apsp_spec_$rep.log)" >> $O/summary.txt
  SHD_PC_TIE_NOSPEC=1 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_nospec_$rep.log 2>&1 || exit 3
  echo "nospec_$rep $(tail -n 1 $O/apsp_nospec_$rep.log)" >> $O/summary.txt
done
