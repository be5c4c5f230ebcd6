#!/bin/bash
# profiles/r02 from one GPU call (compact: raw rocprofv3 traces are reduced
# on the box and deleted, so gpurun_out stays small):
#   bench.json                 the default bench line (N = 1)
#   bench_kernel_stats.csv     rocprofv3 --kernel-trace --stats of the bench (no CPU leg)
#   k_round_pmc_bytes.json     FETCH_SIZE / WRITE_SIZE per k_round_tl dispatch (separate passes)
#   sq_counters.txt            SQ instruction / wait counters per k_round_tl dispatch (two passes)
#   group_kernel_stats.csv     the engine group at one rank (peer-to-peer transport), kernel-trace stats
#   round_timing.txt           phase stamps (timing build, light, no drains)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02
rm -rf $O; mkdir -p $O
ARGS="--steps 2 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py $ARGS > $O/bench_under_rocprof.json 2> $O/trace.err || { tail $O/trace.err; exit 2; }
cp "$(find $O/trace -name '*kernel_stats.csv' | head -1)" $O/bench_kernel_stats.csv && rm -rf $O/trace || exit 2
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
    python3 bench.py $ARGS > $O/fetch_bench.json 2> $O/fetch.err || { tail $O/fetch.err; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
    python3 bench.py $ARGS > $O/write_bench.json 2> $O/write.err || { tail $O/write.err; exit 4; }
python3 scripts/pmc_bytes.py $O/fetch $O/write --fetch-bench $O/fetch_bench.json --write-bench $O/write_bench.json \
    --out $O/k_round_pmc_bytes.json > /dev/null && rm -rf $O/fetch $O/write || exit 5
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_LDS" ; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- \
      python3 bench.py $ARGS > /dev/null 2> $O/pmc$i.err || { tail -5 $O/pmc$i.err; exit 6; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 --kernel k_round_tl > $O/sq_counters.txt && rm -rf $O/pmc1 $O/pmc2 || exit 7
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gtrace -o run -- \
    python3 bench.py --group --exchange p2p $ARGS > $O/group_bench_under_rocprof.json 2> $O/gtrace.err || { tail $O/gtrace.err; exit 8; }
cp "$(find $O/gtrace -name '*kernel_stats.csv' | head -1)" $O/group_kernel_stats.csv && rm -rf $O/gtrace || exit 8
SHD_TIMING_LIGHT=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/round_timing.py --load 16 \
    > $O/round_timing.txt 2>&1 || { tail $O/round_timing.txt; exit 9; }
rm -f $O/*.err
du -sh $O
echo refresh done
