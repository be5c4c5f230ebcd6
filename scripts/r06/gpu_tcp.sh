#!/bin/bash
# round 6: the TCP path's in-call reruns of a contradicted first-touch round (ranked before it runs):
# the TCP GPU tests (one engine and groups), then the mixed-transport bench at 16 384 hosts (round 5:
# first_touch "tables", 49 % of the device rate wall-inclusive) and the echo-only leg beside it
set -o pipefail
O=gpurun_out/r06_tcp
mkdir -p $O
T="timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
$T tests/test_tcp_gpu.py tests/test_tcp_group_gpu.py > $O/tests.log 2>&1 && \
timeout -k 10 600 python3 -u bench.py --workload tcp --tcp-udp --hosts-per-gpu 16384 --steps 2 --warmup 1 \
    --no-cpu-baseline > $O/mixed_16384.json 2> $O/mixed_16384.err && \
timeout -k 10 400 python3 -u bench.py --workload tcp --hosts-per-gpu 16384 --steps 2 --warmup 1 \
    --no-cpu-baseline > $O/echo_16384.json 2> $O/echo_16384.err
