#!/bin/bash
# round 5: SSSP row kernel phase cycles (SHD_SSSP_TIMING build), 10 k vertices
set -o pipefail
O=gpurun_out/r05_sssp
mkdir -p $O
SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvt.so timeout -k 10 120 python -u scripts/sssp_timing.py 10000 > $O/sssp_timing.txt 2>&1
echo "rc=$?"; cat $O/sssp_timing.txt
