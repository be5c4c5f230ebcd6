#!/bin/bash
# round 3: TCP path with vertex-pair path tables and a 2048-packet pool --
# parity tests, the 65 k-host bench line (CPU baseline on its 4096-host
# sample), and rocprof kernel statistics (csv)
set -o pipefail
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tcp_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tcp_tests.log 2>&1 || { tail -30 $O/tcp_tests.log; exit 1; }
tail -2 $O/tcp_tests.log
timeout -k 10 300 python3 bench.py --workload tcp --hosts-per-gpu 4096 --steps 1 --warmup 0 --no-cpu-baseline > $O/tcp_16384.json 2> $O/tcp_16384.err || { tail $O/tcp_16384.err; exit 2; }
cat $O/tcp_16384.json
timeout -k 10 600 python3 bench.py --workload tcp --steps 2 --warmup 1 > $O/tcp_bench.json 2> $O/tcp_bench.err || { tail $O/tcp_bench.err; exit 3; }
cat $O/tcp_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tcp -o tcp -- python3 bench.py --workload tcp --steps 1 --warmup 0 --no-cpu-baseline > $O/tcp_prof_bench.json 2> $O/tcp_prof.err || { tail $O/tcp_prof.err; exit 5; }
find $O/prof_tcp -name "*stats*"
