#!/bin/bash
# round 6: the tied rows' second pass with k_sssp_tie_g's distances (no Bellman-Ford again) against the
# Bellman-Ford again (SHD_PC_TIE_NOGD): tie parity (4-B and 8-B values, and without), the 10 k whole-ms build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tiegd
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests_gd.log 2>&1 || exit 2
SHD_PC_TIE_HV8=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_gd_hv8.log 2>&1 || exit 2
SHD_PC_TIE_NOGD=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_nogd.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_gd_$rep.log 2>&1 || exit 3
  echo "gd_$rep $(tail -n 1 $O/apsp_gd_$rep.log)" >> $O/summary.txt
  SHD_PC_TIE_NOGD=1 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_nogd_$rep.log 2>&1 || exit 3
  echo "nogd_$rep $(tail -n 1 $O/apsp_nogd_$rep.log)" >> $O/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 scripts/r06/tie_once.py > $O/tr.log 2>&1 || exit 4
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv && rm -rf $O/tr
