#!/bin/bash
# round 5: queued frontier depth A/B (SHD_SSSP_BFQ = 1, 2 (default), 4, 8 vertices per half-wave)
set -o pipefail
O=gpurun_out/r05_bfq2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
L=shadow-1_amd
for rep in 1 2; do
  for q in q1 q2 q4 q8; do
    lib=$L/libshdgpu_pcv$q.so; [ $q = q2 ] && lib=$L/libshdgpu.so
    SHDGPU_LIB=$lib timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/${q}_$rep.log 2>&1 || exit 3
    echo "rep $rep $q: $(tail -1 $O/${q}_$rep.log)"
  done
done
for q in q4 q8; do
  SHDGPU_LIB=$L/libshdgpu_pcv$q.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread \
      tests/test_pathcache_gpu.py > $O/tests_$q.log 2>&1; echo "tests $q rc=$?"; tail -1 $O/tests_$q.log
done
