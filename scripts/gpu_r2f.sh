#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
SHD_TIMING_LIGHT=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/round_timing.py --load 16 \
    > gpurun_out/round_timing.txt 2>&1 || { tail gpurun_out/round_timing.txt; exit 1; }
cat gpurun_out/round_timing.txt | grep -v amdgpu.ids
timeout -k 10 600 python bench.py --workload c4 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
