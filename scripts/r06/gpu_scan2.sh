#!/bin/bash
# round 6: the sparse scan with each lane's idle bound, shared with the group's sparse round
# (k_round_spx); the p2p mapping self-check; bench.py's N > 1 parity leg; the restore point renewed
# between batches; the TCP same-window connect refusal.  Parity first, then the C5-shard bench twice
# (one engine) and once through the one-rank group, the stamps and the event-path counters at 3 s
set -o pipefail
O=gpurun_out/r06_scan2
mkdir -p $O
T="timeout -k 10 1200 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
$T tests/test_engine_gpu.py > $O/tests_engine.log 2>&1 && \
$T tests/test_tcp_gpu.py -k "refuses" > $O/tests_tcp.log 2>&1 && \
$T tests/test_bench_parity_gpu.py tests/test_xgroup_procs_gpu.py > $O/tests_group.log 2>&1 && \
$T tests/test_fullsize_gpu.py > $O/tests_full.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline \
    > $O/bench_c5_$r.json 2> $O/bench_c5_$r.err || exit 3
done && \
timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline \
    --group > $O/bench_c5_group.json 2> $O/bench_c5_group.err && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 3.0 > $O/c5_nowait_3s.txt 2>&1 && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_cnt.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 3.0 > $O/c5_counts_3s.txt 2>&1
