#!/bin/bash
# round 6: phase stamps of the lean persistent rounds (C3 headline k_round_ps, the C5 shard k_round_sp at
# 3 s) and the bench lines of the same tree
set -o pipefail
O=gpurun_out/r06_stamps2
mkdir -p $O
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py \
    > $O/c3_nowait.txt 2>&1 && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 3.0 > $O/c5_nowait_3s.txt 2>&1 && \
timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 --steps 4 --warmup 2 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 \
    > $O/c5.json 2> $O/c5.err
