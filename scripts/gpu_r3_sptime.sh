#!/bin/bash
# round 3: phase stamps of k_round_sp on the C5 shard, and of k_round_ps on C3
set -o pipefail
O=gpurun_out/r03/sp
mkdir -p $O
export SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so
timeout -k 10 300 python3 scripts/ps_timing.py --workload c5 --hosts 125000 > $O/sp_timing_c5.txt 2>&1 || { tail $O/sp_timing_c5.txt; exit 1; }
cat $O/sp_timing_c5.txt
