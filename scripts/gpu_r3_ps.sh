#!/bin/bash
# round 3: the persistent round kernel -- parity suites, then the bench (ps on / off)
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_engine_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py tests/test_pathcache_gpu.py \
    > gpurun_out/r03/ps_tests.log 2>&1 || { tail -30 gpurun_out/r03/ps_tests.log; exit 1; }
tail -3 gpurun_out/r03/ps_tests.log
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r03/bench_ps.json 2> gpurun_out/r03/bench_ps.err || { tail gpurun_out/r03/bench_ps.err; exit 2; }
SHD_NO_PS=1 timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r03/bench_tl.json 2> gpurun_out/r03/bench_tl.err || { tail gpurun_out/r03/bench_tl.err; exit 3; }
python3 -c "
import json
for f in ('bench_ps','bench_tl'):
    d=json.loads(open('gpurun_out/r03/%s.json'%f).read().strip().splitlines()[-1])
    print(f, round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms/step', d.get('roofline',{}).get('achieved'))
"
