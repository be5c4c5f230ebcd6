#!/bin/bash
# profiles/r06 (C3 headline) from one GPU call; raw traces reduced on the box:
#   bench.json              bench.py defaults (C3 headline, CPU baseline on the same window)
#   timed_region.json       rocprofv3 --kernel-trace --marker-trace: round kernel time inside bench's timed region
#   bench_kernel_stats.csv  the same run's --stats summary (whole run)
#   pmc_calibration.json    FETCH_SIZE / WRITE_SIZE against known bytes (scripts/microbench/pmc_calib.hip)
#   pmc_traffic.json        FETCH_SIZE x correction + WRITE_SIZE per round over the timed region (separate passes;
#                           C3's k_round_ps and the C5 shard's k_round_sp)
#   sq_counters.txt         SQ counters of k_round_ps (two passes; per dispatch = one persistent batch)
#   barrier.txt, launch.txt the seam microbenchmarks
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p
rm -rf $O; mkdir -p $O
ARGS="--steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
echo bench ok
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 bench.py $ARGS > $O/bench_rocprof.json 2> $O/tr.err || { tail $O/tr.err; exit 2; }
python3 scripts/rocprof_timed.py $O/tr $O/bench_rocprof.json --out $O/timed_region.json > /dev/null || exit 3
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/bench_kernel_stats.csv && rm -rf $O/tr || exit 3
echo trace ok
timeout -k 10 60 ./scripts/microbench/pmc_calib > $O/pmc_calib_known.json 2>&1 || exit 4
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calf -o run -- ./scripts/microbench/pmc_calib > /dev/null 2> $O/calf.err || { tail -5 $O/calf.err; exit 4; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calw -o run -- ./scripts/microbench/pmc_calib > /dev/null 2> $O/calw.err || { tail -5 $O/calw.err; exit 4; }
python3 scripts/pmc_calib.py $O/calf $O/calw $O/pmc_calib_known.json --out $O/pmc_calibration.json > /dev/null && rm -rf $O/calf $O/calw || exit 4
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
    python3 bench.py $ARGS > $O/fetch_bench.json 2> $O/fetch.err || { tail $O/fetch.err; exit 5; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
    python3 bench.py $ARGS > $O/write_bench.json 2> $O/write.err || { tail $O/write.err; exit 6; }
python3 scripts/pmc_traffic.py $O/fetch $O/write $O/fetch_bench.json $O/write_bench.json $O/pmc_calibration.json \
    --key c3-10000h/k_round_ps --out $O/pmc_traffic.json && rm -rf $O/fetch $O/write || exit 7
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
