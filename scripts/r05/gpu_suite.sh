#!/bin/bash
# round 5: the whole GPU suite (no -x: every failure listed), smoke(), and the
# two-row kernel's queue depth A/B (SHD_SSSP_BFQ2 = 1 default, 2 variant)
set -o pipefail
O=gpurun_out/r05_suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -30
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $O/smoke.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/q21_$rep.log 2>&1 || exit 3
  SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvq22.so timeout -k 10 200 python -u scripts/r05/apsp_ties.py > $O/q22_$rep.log 2>&1 || exit 4
  for k in q21 q22; do echo "rep $rep $k: $(tail -1 $O/${k}_$rep.log)"; done
done
