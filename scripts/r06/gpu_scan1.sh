#!/bin/bash
# round 6: the sparse scan's idle-host bound from the OR of the bitmaps -- parity (forced-sparse and
# the C5 / C3 full-size fixtures), the C5-shard bench twice, and the stamps at 3 s
set -o pipefail
O=gpurun_out/r06_scan1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_engine_gpu.py -k "sparse" > $O/tests_engine.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_fullsize_gpu.py -k "c5 or c3_full" > $O/tests_full.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline \
    > $O/bench_c5_$r.json 2> $O/bench_c5_$r.err || exit 3
done && \
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim_p0nw.so timeout -k 10 300 python3 -u scripts/ps_timing.py --workload c5 \
    --hosts 125000 --at 3.0 > $O/c5_nowait_3s.txt 2>&1
