#!/bin/bash
# round 5: the two-row kernel's rows in one queue (default) against a queue per row
set -o pipefail
O=gpurun_out/r05_mixq
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvsepq.so timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/sep_$rep.log 2>&1 || exit 3
  timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/mix_$rep.log 2>&1 || exit 4
  for k in sep mix; do echo "rep $rep $k: $(tail -1 $O/${k}_$rep.log)"; done
done
