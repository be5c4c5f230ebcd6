#!/bin/bash
# round 4: the TCP tests on the final TCP path, then its bench under
# rocprofv3 --kernel-trace --stats (the round kernel's dispatch times)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_tcpfinal
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tcp_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 bench.py --workload tcp --no-cpu-baseline --steps 1 --warmup 0 > $O/tcp_bench.json 2> $O/tr.err || { tail -5 $O/tr.err; exit 2; }
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/tcp_kernel_stats.csv && rm -rf $O/tr || exit 3
head -5 $O/tcp_kernel_stats.csv; tail -1 $O/tcp_bench.json | cut -c1-200
