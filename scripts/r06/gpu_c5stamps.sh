#!/bin/bash
# round 6: faithful phase stamps of the sparse persistent round (k_round_sp) at the north star's per-GPU
# shard (C5, 125 k hosts): the timing build keeps the product's one parameter copy per batch
# (SHD_TIMING_P0); issue-point (nowait) and drained stamps, at 2 s and 3 s; the product's bench beside
set -o pipefail
O=gpurun_out/r06_c5stamps
mkdir -p $O
timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline \
    > $O/bench_c5.json 2> $O/bench_c5.err && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 2.0 > $O/c5_nowait_2s.txt 2>&1 && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 3.0 > $O/c5_nowait_3s.txt 2>&1 && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 3.0 > $O/c5_light_3s.txt 2>&1 && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py \
    > $O/c3_nowait.txt 2>&1
