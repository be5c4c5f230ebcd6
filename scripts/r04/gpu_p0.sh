#!/bin/bash
# round 4: one parameter copy per persistent batch (A) against a copy per round
# (B, libshdgpu_var.so built with -DSHD_PS_PR), C3 and the C5 shard; the
# one-cache co-simulation tests first
set -o pipefail
O=gpurun_out/r04_p0
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ingress_gpu.py tests/test_pc_touches_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/ingress.log 2>&1; echo "ingress rc=$?"; grep -E "PASSED|FAILED|Error|passed|failed" $O/ingress.log | tail -15
: > $O/ab.log
for k in 0 1 2; do
  for v in A B; do
    if [ $v = B ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_var.so; else unset SHDGPU_LIB; fi
    timeout -k 10 150 python bench.py --no-cpu-baseline --lossy-edge-loss-max 0 > $O/ab_$v$k.json 2> $O/ab_$v$k.err || { tail -5 $O/ab_$v$k.err; exit 2; }
    python3 -c "import json; d=json.load(open('$O/ab_$v$k.json')); print('$v', round(d['value']/1e6,2), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])" | tee -a $O/ab.log
  done
done
for v in A B; do
  if [ $v = B ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_var.so; else unset SHDGPU_LIB; fi
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 3; }
  python3 -c "import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c5 $v', round(d['value']/1e6,2), r['kernel'], r['avg_round_us'])" | tee -a $O/ab.log
done
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/ps_timing.py > $O/timing_c3.txt 2>&1 || { tail -5 $O/timing_c3.txt; exit 4; }
cat $O/timing_c3.txt
# APSP: Gauss-Seidel sweeps (libshdgpu_pcvgs.so, -DSHD_SSSP_GS) against the product; parity of the variant
for lib in libshdgpu.so libshdgpu_pcvgs.so; do
  SHDGPU_LIB=shadow-1_amd/$lib timeout -k 10 120 python -u scripts/apsp_timing.py > $O/apsp_$lib.json 2> $O/apsp_$lib.err || { tail $O/apsp_$lib.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/apsp_$lib.json'));print('$lib', {k:(v['ms'],v.get('sssp_ms'),v.get('iters')) for k,v in d.items()})"
done
SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvgs.so timeout -k 10 300 python -u -m pytest tests/test_pathcache_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pc_gs.log 2>&1; echo "pathcache gs rc=$?"; tail -3 $O/pc_gs.log
# TCP: the mailbox part counters of round 3's 881351e (libshdgpu_tcpv.so, -DSHD_TCP_PARTS) against the
# product, 65 536 hosts; per-dispatch k_tcp_round durations from a kernel trace of each
timeout -k 10 300 python -u -m pytest tests/test_tcp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tcp_tests.log 2>&1; echo "tcp tests rc=$?"; tail -2 $O/tcp_tests.log
SHDGPU_LIB=shadow-1_amd/libshdgpu_tcpv.so timeout -k 10 300 python -u -m pytest tests/test_tcp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tcpv_tests.log 2>&1; echo "tcpv tests rc=$?"; tail -2 $O/tcpv_tests.log
for v in A B; do
  if [ $v = B ]; then L=shadow-1_amd/libshdgpu_tcpv.so; else L=shadow-1_amd/libshdgpu.so; fi
  SHDGPU_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_tcp_$v -o tcp -- python3 bench.py --workload tcp --steps 1 --warmup 0 --no-cpu-baseline > $O/tcp_$v.json 2> $O/tcp_$v.err || { tail -5 $O/tcp_$v.err; exit 6; }
  python3 -c "import json; d=json.loads(open('$O/tcp_$v.json').read().strip().splitlines()[-1]); print('tcp $v', round(d['value']/1e6,2), d.get('wall_inclusive'))"
done
