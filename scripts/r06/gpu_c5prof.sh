#!/bin/bash
# round 6: the north star's per-GPU shard (C5 model, 125 k hosts) under rocprofv3 on the final engine: kernel
# stats of the whole run and k_round_sp over bench.py's timed region; (its C4 and C3-100k lines ran with one warm-up step: see gpu_c4.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_c5prof
rm -rf $O; mkdir -p $O
C5="--workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 bench.py $C5 > $O/c5_rocprof.json 2> $O/tr.err || { tail $O/tr.err; exit 1; }
python3 scripts/rocprof_timed.py $O/tr $O/c5_rocprof.json --out $O/c5_timed_region.json > /dev/null || exit 2
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/c5_kernel_stats.csv && rm -rf $O/tr || exit 2
timeout -k 10 400 python3 bench.py --workload c4 --no-cpu-baseline --steps 2 --warmup 1 > $O/c4.json 2> $O/c4.err || exit 3
timeout -k 10 400 python3 bench.py --hosts-per-gpu 100000 --no-cpu-baseline --lossy-edge-loss-max 0 --steps 2 --warmup 1 \
    > $O/c3_100k.json 2> $O/c3_100k.err || exit 4
rm -f $O/*.err
