#!/bin/bash
# round 3: per-phase clocks of the round kernel (prof build) on C4 and the C5 shard
set -o pipefail
O=gpurun_out/r03/prof
mkdir -p $O
export SHDGPU_LIB=shadow-1_amd/libshdgpu_prof.so
timeout -k 10 300 python3 scripts/prof_round.py --workload c4 > $O/c4.txt 2>&1 || { tail $O/c4.txt; exit 1; }
cat $O/c4.txt
timeout -k 10 300 python3 scripts/prof_round.py --workload c5 --hosts 125000 > $O/c5.txt 2>&1 || { tail $O/c5.txt; exit 1; }
cat $O/c5.txt
