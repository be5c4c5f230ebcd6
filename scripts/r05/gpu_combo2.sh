#!/bin/bash
# round 5: path-cache + TCP tests, LDS arc offsets A/B on the APSP build
# (SHD_PC_NO_LDS_OFF), TCP bench with the kept workspace
set -o pipefail
O=gpurun_out/r05_combo2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_pathcache_gpu.py \
    tests/test_tcp_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1; do
  SHD_PC_NO_LDS_OFF=1 timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/apsp_glb_$rep.log 2>&1 || exit 3
  timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/apsp_lds_$rep.log 2>&1 || exit 4
  echo "rep $rep global-offsets: $(tail -1 $O/apsp_glb_$rep.log)"
  echo "rep $rep lds-offsets:    $(tail -1 $O/apsp_lds_$rep.log)"
done
timeout -k 10 900 python -u bench.py --workload tcp --steps 3 --warmup 1 > $O/tcp_bench.json 2> $O/tcp_bench.err
echo "tcp bench rc=$?"; tail -3 $O/tcp_bench.err; cat $O/tcp_bench.json
