#!/bin/bash
# round 3: persistent-round phase stamps, barrier microbench, PMC calibration,
# rocprof timed-region check of the bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 60 ./scripts/microbench/barrier > $O/barrier.txt 2>&1 || { cat $O/barrier.txt; exit 1; }
cat $O/barrier.txt
SHD_TIMING_LIGHT=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/ps_timing.py > $O/ps_timing.txt 2>&1 || { tail $O/ps_timing.txt; exit 2; }
cat $O/ps_timing.txt
timeout -k 10 60 ./scripts/microbench/pmc_calib > $O/pmc_calib_known.json 2>&1 || exit 3
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calf -o run -- ./scripts/microbench/pmc_calib > /dev/null 2> $O/calf.err || { tail -5 $O/calf.err; exit 4; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calw -o run -- ./scripts/microbench/pmc_calib > /dev/null 2> $O/calw.err || { tail -5 $O/calw.err; exit 5; }
python3 scripts/pmc_calib.py $O/calf $O/calw $O/pmc_calib_known.json --out $O/pmc_calibration.json && rm -rf $O/calf $O/calw || exit 6
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 > $O/bench_rocprof.json 2> $O/tr.err || { tail $O/tr.err; exit 7; }
python3 scripts/rocprof_timed.py $O/tr $O/bench_rocprof.json --out $O/timed_region.json || exit 8
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/bench_kernel_stats.csv; rm -rf $O/tr
echo done
