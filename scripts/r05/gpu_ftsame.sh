#!/bin/bash
# the TCP path's device first touches accepting contradicted choices whose candidates give the same bits:
# every TCP test (one engine, groups), the mixed bench leg at 16 384 hosts
set -o pipefail
O=gpurun_out/r05_ftsame
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_tcp_gpu.py tests/test_tcp_group_gpu.py -v --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
grep -E "FAILED|passed|failed" $O/tests.log | tail -30
timeout -k 10 900 python -u bench.py --workload tcp --tcp-udp --hosts-per-gpu 16384 --steps 2 --warmup 1 \
    --no-cpu-baseline > $O/mixed_16384.json 2> $O/mixed_16384.err; echo "bench rc=$?"
