#!/bin/bash
# round 3: TCP path v2 (device-side windows, graph-batched rounds, per-destination
# mail lists) -- its parity tests first, then the whole GPU suite, the default
# bench line, the TCP bench line and its rocprof kernel statistics
set -o pipefail
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tcp_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tcp_tests.log 2>&1 || { tail -30 $O/tcp_tests.log; exit 1; }
tail -2 $O/tcp_tests.log
timeout -k 10 300 python3 bench.py --workload tcp --hosts-per-gpu 512 --steps 1 --warmup 0 --no-cpu-baseline > $O/tcp_bench512.json 2> $O/tcp_bench512.err || { tail $O/tcp_bench512.err; exit 2; }
cat $O/tcp_bench512.json
timeout -k 10 600 python3 bench.py --workload tcp --steps 2 --warmup 1 > $O/tcp_bench.json 2> $O/tcp_bench.err || { tail $O/tcp_bench.err; exit 2; }
cat $O/tcp_bench.json
for L in 1 4 16; do
  SHD_TCP_LANES=$L timeout -k 10 300 python3 bench.py --workload tcp --steps 1 --warmup 1 --no-cpu-baseline > $O/tcp_lanes$L.json 2> $O/tcp_lanes$L.err || { tail $O/tcp_lanes$L.err; exit 6; }
  echo lanes $L; cat $O/tcp_lanes$L.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 4; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_tcp -o tcp -- python3 bench.py --workload tcp --steps 1 --warmup 0 --no-cpu-baseline > $O/tcp_prof_bench.json 2> $O/tcp_prof.err || { tail $O/tcp_prof.err; exit 5; }
find $O/prof_tcp -name "*stats*" | head
