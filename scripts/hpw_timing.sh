#!/bin/bash
# round timing (timing build) at several hosts-per-wave settings
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/hpw_timing.log
for h in 64 16 4; do
  echo "== hpw $h" >> gpurun_out/hpw_timing.log
  SHD_HPW=$h SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 150 python scripts/round_timing.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/hpw_timing.log || exit 1
done
cat gpurun_out/hpw_timing.log
