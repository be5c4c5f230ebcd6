#!/bin/bash
# round 4: path prediction -- the GPU suite, the headline A/B (default library
# vs libshdgpu_var.so built with -DSHD_NO_PP), then the phase stamps of the
# timing build (-DSHD_TIMING_LIGHT -DSHD_TIMING_NOWAIT)
set -o pipefail
O=gpurun_out/r04_pp2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_fullsize_gpu.py tests/test_ref_loop_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
: > $O/ab.log
for k in 0 1 2; do
  for v in A B; do
    if [ $v = B ]; then export SHDGPU_LIB=shadow-1_amd/libshdgpu_var.so; else unset SHDGPU_LIB; fi
    timeout -k 10 150 python bench.py --no-cpu-baseline --lossy-edge-loss-max 0 > $O/ab_$v$k.json 2> $O/ab_$v$k.err || { tail -5 $O/ab_$v$k.err; exit 2; }
    python3 -c "import json; d=json.load(open('$O/ab_$v$k.json')); print('$v', round(d['value']/1e6,2), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])" | tee -a $O/ab.log
  done
done
unset SHDGPU_LIB
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/ps_timing.py > $O/timing_c3.txt 2>&1 || { tail -5 $O/timing_c3.txt; exit 3; }
cat $O/timing_c3.txt
