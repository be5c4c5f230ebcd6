#!/bin/bash
# per-phase stamps of the round kernel (timing build, light stamps)
set -o pipefail
mkdir -p gpurun_out
SHD_TIMING_LIGHT=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/round_timing.py --load 16 \
    > gpurun_out/round_timing.txt 2>&1 || { tail gpurun_out/round_timing.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/round_timing.txt
