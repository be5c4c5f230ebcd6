#!/bin/bash
# round 5: APSP A/B -- spatial relabelling x flattened frontier arcs; the path
# cache's GPU tests on the default build first
set -o pipefail
O=gpurun_out/r05_apsp
mkdir -p $O
timeout -k 10 10 true \
    > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
  echo "== default (relabel + flat)"; timeout -k 10 300 python -u scripts/r05/apsp_ties.py 2>&1 | tail -1
  echo "== no relabel, flat"; SHD_PC_NO_RELABEL=1 timeout -k 10 300 python -u scripts/r05/apsp_ties.py 2>&1 | tail -1
  echo "== relabel, pairs"; SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvpairs.so timeout -k 10 300 python -u scripts/r05/apsp_ties.py 2>&1 | tail -1
  echo "== no relabel, pairs (round 4)"; SHD_PC_NO_RELABEL=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvpairs.so timeout -k 10 300 python -u scripts/r05/apsp_ties.py 2>&1 | tail -1
done 2>&1 | tee $O/ab.log
SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvt.so timeout -k 10 120 python -u scripts/sssp_timing.py 10000 > $O/sssp_timing.txt 2>&1
SHD_PC_NO_RELABEL=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvt.so timeout -k 10 120 python -u scripts/sssp_timing.py 10000 > $O/sssp_timing_norelabel.txt 2>&1
cat $O/sssp_timing.txt $O/sssp_timing_norelabel.txt
