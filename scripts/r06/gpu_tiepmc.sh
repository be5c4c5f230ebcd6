#!/bin/bash
# round 6: SQ counters and the kernel trace of k_sssp_tie_g on the 10 k whole-ms build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tiepmc
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 scripts/r06/tie_once.py > $O/tr.log 2>&1 || exit 1
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv && rm -rf $O/tr || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_FLAT SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- \
      python3 scripts/r06/tie_once.py > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 2; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 $O/pmc3 --kernel k_sssp_tie_g > $O/sq_counters.txt && rm -rf $O/pmc1 $O/pmc2 $O/pmc3
