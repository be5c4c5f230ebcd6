#!/bin/bash
# phase stamps of the sparse persistent round (k_round_sp) at the north star's per-GPU shard (C5, 125 k
# hosts): drained stamps (SHD_TIMING_LIGHT) and issue-point stamps (+ SHD_TIMING_NOWAIT); C3 beside
set -o pipefail
mkdir -p gpurun_out/r05_c5phases
SHD_SP_HOSTS=512 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_light.so timeout -k 10 300 python -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 > gpurun_out/r05_c5phases/c5_light.txt 2>&1 && \
SHD_SP_HOSTS=512 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_nowait.so timeout -k 10 300 python -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 > gpurun_out/r05_c5phases/c5_nowait.txt 2>&1 && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_nowait.so timeout -k 10 300 python -u scripts/ps_timing.py \
    > gpurun_out/r05_c5phases/c3_nowait.txt 2>&1
