#!/bin/bash
# profiles/r06, second call: the C5 shard's PMC traffic (merged into refresh_r06a's pmc_traffic.json, copied
# to profiles/r06 between the calls), SQ counters of k_round_ps, the seam microbenchmarks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06pb
rm -rf $O; mkdir -p $O
cp profiles/r06/pmc_calibration.json profiles/r06/pmc_traffic.json $O/ || exit 1
ARGS="--steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
# the north star's per-GPU shard (C5, 125 k hosts, k_round_sp): its traffic too
C5="--workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch5 -o run -- \
    python3 bench.py $C5 > $O/fetch_c5.json 2> $O/fetch5.err || { tail $O/fetch5.err; exit 5; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write5 -o run -- \
    python3 bench.py $C5 > $O/write_c5.json 2> $O/write5.err || { tail $O/write5.err; exit 6; }
python3 scripts/pmc_traffic.py $O/fetch5 $O/write5 $O/fetch_c5.json $O/write_c5.json $O/pmc_calibration.json \
    --key c5-125000h/k_round_sp --out $O/pmc_traffic.json && rm -rf $O/fetch5 $O/write5 || exit 7
echo pmc ok
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_LDS" ; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- \
      python3 bench.py $ARGS > /dev/null 2> $O/pmc$i.err || { tail -5 $O/pmc$i.err; exit 8; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 --kernel k_round_ps > $O/sq_counters.txt && rm -rf $O/pmc1 $O/pmc2 || exit 9
echo sq ok

timeout -k 10 60 ./scripts/microbench/barrier > $O/barrier.txt 2>&1 || exit 11
timeout -k 10 60 ./scripts/microbench/launch > $O/launch.txt 2>&1 || exit 12
rm -f $O/*.err
echo refresh done
