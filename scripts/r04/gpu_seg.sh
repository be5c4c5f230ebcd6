#!/bin/bash
# round 4: loop segment timing (C3, C5 forced sparse) and the one-cache co-simulation tests
set -o pipefail
O=gpurun_out/r04_seg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ingress_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not bridged" > $O/ingress.log 2>&1; echo "ingress rc=$?"; tail -15 $O/ingress.log
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/ps_timing.py > $O/timing_c3.txt 2>&1 || { tail -5 $O/timing_c3.txt; exit 3; }
cat $O/timing_c3.txt
SHD_SP_HOSTS=512 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 300 python3 scripts/ps_timing.py --workload c5 --hosts 125000 > $O/timing_c5.txt 2>&1 || { tail -5 $O/timing_c5.txt; exit 4; }
cat $O/timing_c5.txt
