#!/bin/bash
# round 3: persistent rounds, second pass -- parity, bench at 64 / 32 hosts per wave, phase stamps
set -o pipefail
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_engine_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py \
    > $O/ps2_tests.log 2>&1 || { tail -30 $O/ps2_tests.log; exit 1; }
tail -2 $O/ps2_tests.log
for v in 64 32; do
  SHD_HPW=$v timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 > $O/bench_ps2_h$v.json 2> $O/bench_ps2_h$v.err || { tail $O/bench_ps2_h$v.err; exit 2; }
done
python3 -c "
import json
for v in (64, 32):
    d=json.loads(open('gpurun_out/r03/bench_ps2_h%d.json'%v).read().strip().splitlines()[-1])
    r=d['roofline']
    print('hpw', v, round(d['value']/1e6,2), 'M', r['kernel'], r['avg_round_us'], 'us/round', r['avg_in_kernel_us'], 'in-kernel', d['timed_batches_persistent'], 'ps batches')
"
SHD_TIMING_LIGHT=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/ps_timing.py > $O/ps_timing2.txt 2>&1 || { tail $O/ps_timing2.txt; exit 3; }
cat $O/ps_timing2.txt
