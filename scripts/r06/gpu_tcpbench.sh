#!/bin/bash
# round 6, final tree: the TCP echo bench (65 536 hosts) and the mixed-transport bench (16 384 hosts)
set -o pipefail
O=gpurun_out/r06_tcpbench
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 bench.py --workload tcp --no-cpu-baseline > $O/tcp.json 2> $O/tcp.err || exit 1
timeout -k 10 600 python3 bench.py --workload tcp --tcp-udp --hosts-per-gpu 16384 --steps 2 --warmup 1 --no-cpu-baseline > $O/mixed.json 2> $O/mixed.err || exit 2
rm -f $O/*.err
