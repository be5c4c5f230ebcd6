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
