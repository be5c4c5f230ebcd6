#!/bin/bash
# round 6: SQ counters of the TCP round kernel (k_tcp_round) on the bench's TCP echo model (65 536 hosts)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tcppmc
rm -rf $O; mkdir -p $O
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- \
      python3 bench.py --workload tcp --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 4; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 --kernel k_tcp_round > $O/sq_counters.txt && rm -rf $O/pmc1 $O/pmc2
