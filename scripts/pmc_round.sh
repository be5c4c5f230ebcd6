#!/bin/bash
# SQ counters of the round kernel (one counter set per rocprofv3 pass)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 1 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_LDS" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc$i -o run -- \
      python3 bench.py $ARGS > /dev/null 2> gpurun_out/pmc$i.err || { echo "pass $i failed"; tail -5 gpurun_out/pmc$i.err; exit $i; }
done
echo pmc done
