#!/bin/bash
# round 4: where a TCP round's time goes -- per-step cycles per lane and each
# round's busiest lane (libshdgpu_tcpv.so built with -DSHD_TCP_PROF), at 65 536 hosts
set -o pipefail
O=gpurun_out/r04_tcpprof${1:-}
mkdir -p $O
SHDGPU_LIB=shadow-1_amd/libshdgpu_tcpv.so timeout -k 10 300 python bench.py --workload tcp --no-cpu-baseline --steps 1 --warmup 0 > $O/bench.json 2> $O/prof.txt; echo "rc=$?"
grep -c tcp_round $O/prof.txt; grep tcp_prof $O/prof.txt | head -40
