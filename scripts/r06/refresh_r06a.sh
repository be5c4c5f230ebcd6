#!/bin/bash
# profiles/r06 (C3 headline) from one GPU call; raw traces reduced on the box:
#   bench.json              bench.py defaults (C3 headline, CPU baseline on the same window)
#   timed_region.json       rocprofv3 --kernel-trace --marker-trace: round kernel time inside bench's timed region
#   bench_kernel_stats.csv  the same run's --stats summary (whole run)
#   pmc_calibration.json    FETCH_SIZE / WRITE_SIZE against known bytes (scripts/microbench/pmc_calib.hip)
#   pmc_traffic.json        FETCH_SIZE x correction + WRITE_SIZE per round over the timed region (separate passes;
#                           C3's k_round_ps and the C5 shard's k_round_sp)
#   (refresh_r06b.sh: the C5 shard's traffic, SQ counters, the seam microbenchmarks)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06pa
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
echo pmc ok
echo refresh a done
