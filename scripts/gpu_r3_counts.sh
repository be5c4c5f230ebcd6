#!/bin/bash
# round 3: event-path counters (C5 shard, C4, C3) and no-drain phase stamps of k_round_sp on the C5 shard
set -o pipefail
O=gpurun_out/r03/counts
mkdir -p $O
for w in "c5 --hosts 125000" "c4" "c3"; do
  SHDGPU_LIB=shadow-1_amd/libshdgpu_cnt.so timeout -k 10 300 python3 scripts/event_counts.py --workload $w >> $O/counts.txt 2>&1 || { tail $O/counts.txt; exit 1; }
done
grep -v amdgpu.ids $O/counts.txt
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 300 python3 scripts/ps_timing.py --workload c5 --hosts 125000 > $O/sp_timing_nowait.txt 2>&1 || { tail $O/sp_timing_nowait.txt; exit 1; }
grep -v amdgpu.ids $O/sp_timing_nowait.txt
