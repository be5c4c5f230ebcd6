#!/bin/bash
# round 5: SQ counters of the two-row SSSP kernel (two passes, one run each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_apsppmc
mkdir -p $O
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- python3 scripts/r05/apsp_once.py \
      > $O/pmc$i.out 2> $O/pmc$i.err || { tail -5 $O/pmc$i.err; exit 8; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 --kernel k_sssp_rows2_lds > $O/sq_counters.txt && rm -rf $O/pmc1 $O/pmc2 || exit 9
cat $O/sq_counters.txt
