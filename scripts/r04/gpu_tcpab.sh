#!/bin/bash
# round 4: a TCP change (A: libshdgpu.so) against the previous code (B:
# libshdgpu_tcpv.so built from it, TCP_SRC=...; C: libshdgpu_tcpc.so if present,
# a third build), the TCP tests first; the
# bench at 65 536 hosts, two alternations
set -o pipefail
O=gpurun_out/r04_tcpab${1:-}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tcp_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
: > $O/ab.log
for k in 0 1; do
  for v in A B C; do
    unset SHDGPU_LIB
    if [ $v = B ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_tcpv.so; fi
    if [ $v = C ]; then [ -f shadow-1_amd/libshdgpu_tcpc.so ] || continue; export SHDGPU_LIB=shadow-1_amd/libshdgpu_tcpc.so; fi
    timeout -k 10 200 python bench.py --workload tcp --no-cpu-baseline --steps 1 --warmup 0 > $O/tcp_$v$k.json 2> $O/tcp_$v$k.err || { tail -5 $O/tcp_$v$k.err; exit 2; }
    python3 -c "import json; d=json.loads(open('$O/tcp_$v$k.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), d['roofline']['avg_round_us'], d['wall_inclusive']['value'], d['wall_s'])" | tee -a $O/ab.log
  done
done
