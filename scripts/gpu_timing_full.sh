#!/bin/bash
# per-event-class cycle costs of the round kernel (timing build, full stamps)
set -o pipefail
mkdir -p gpurun_out
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/round_timing.py --load 16 \
    > gpurun_out/round_timing_full.txt 2>&1 || { tail gpurun_out/round_timing_full.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/round_timing_full.txt
