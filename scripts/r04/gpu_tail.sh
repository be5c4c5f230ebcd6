#!/bin/bash
# round 4: the refresh's last steps (the persistent round's phase stamps, the
# seam microbenchmarks), then the TCP A/B/C of gpu_tcpab.sh
set -o pipefail
O=gpurun_out/r04p2
mkdir -p $O
SHD_TIMING_LIGHT=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/ps_timing.py > $O/ps_timing.txt 2>&1 || { tail $O/ps_timing.txt; exit 10; }
timeout -k 10 60 ./scripts/microbench/barrier > $O/barrier.txt 2>&1 || exit 11
timeout -k 10 60 ./scripts/microbench/launch > $O/launch.txt 2>&1 || exit 12
echo tail ok
bash scripts/r04/gpu_tcpab.sh 5
