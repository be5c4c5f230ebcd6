#!/bin/bash
# round 6: k_sssp_tie_g's sifts in VALU with uniform exits (VH) against the scalarized sifts (SHD_PC_TIE_SHEAP),
# both with every chunk's loads through one register set: tie parity both ways (4-B and 8-B values), the 10 k
# whole-ms build two alternations, then the SQ counters of the VH kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tievh
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py > $O/tests_vh.log 2>&1 || exit 2
SHD_PC_TIE_HV8=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_vh_hv8.log 2>&1 || exit 2
SHD_PC_TIE_SHEAP=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_pathcache_gpu.py -k tie > $O/tests_sheap.log 2>&1 || exit 2
for rep in 1 2; do
  timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_vh_$rep.log 2>&1 || exit 3
  echo "vh_$rep $(tail -n 1 $O/apsp_vh_$rep.log)" >> $O/summary.txt
  SHD_PC_TIE_SHEAP=1 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_sheap_$rep.log 2>&1 || exit 3
  echo "sheap_$rep $(tail -n 1 $O/apsp_sheap_$rep.log)" >> $O/summary.txt
done
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- \
      python3 scripts/r06/tie_once.py > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 4; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 --kernel k_sssp_tie_g > $O/sq_counters.txt && rm -rf $O/pmc1 $O/pmc2
