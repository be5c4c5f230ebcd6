#!/bin/bash
# per-batch activity (SHD_SP_VERBOSE) of C5's shard and C4, sparse throughout and dense throughout
set -o pipefail
O=gpurun_out/r05_spverb
mkdir -p $O
export SHD_SP_VERBOSE=1
SHD_SP_DENSE_FRAC=2 timeout -k 10 300 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline > $O/c5_sp.json 2> $O/c5_sp.err &&
SHD_SP_DENSE_FRAC=0 timeout -k 10 300 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline > $O/c5_tl.json 2> $O/c5_tl.err &&
SHD_SP_DENSE_FRAC=2 timeout -k 10 300 python3 bench.py --workload c4 --steps 2 --warmup 2 --no-cpu-baseline > $O/c4_sp.json 2> $O/c4_sp.err &&
SHD_SP_DENSE_FRAC=0 timeout -k 10 300 python3 bench.py --workload c4 --steps 2 --warmup 2 --no-cpu-baseline > $O/c4_tl.json 2> $O/c4_tl.err &&
SHD_SP_DENSE_FRAC=2 timeout -k 10 300 python3 bench.py --workload c3 --hosts-per-gpu 100000 --steps 2 --warmup 2 --no-cpu-baseline > $O/c3h_sp.json 2> $O/c3h_sp.err &&
SHD_SP_DENSE_FRAC=0 timeout -k 10 300 python3 bench.py --workload c3 --hosts-per-gpu 100000 --steps 2 --warmup 2 --no-cpu-baseline > $O/c3h_tl.json 2> $O/c3h_tl.err
rc=$?; echo rc=$rc; grep -c "shd: batch" $O/*.err
