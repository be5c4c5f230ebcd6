#!/bin/bash
# round 6: k_round_sp's scan split (first batch's words landed, compaction done) at the C5 shard, 3 s
set -o pipefail
O=gpurun_out/r06_c5scan
mkdir -p $O
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 3.0 > $O/c5_nowait_3s.txt 2>&1
