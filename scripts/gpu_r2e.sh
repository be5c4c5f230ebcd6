#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
SHD_TL_STRICT=1 timeout -k 10 200 python -u scripts/hpw_probe.py 64 > gpurun_out/tl_strict.log 2>&1 || { tail gpurun_out/tl_strict.log; exit 1; }
timeout -k 10 200 python -u scripts/hpw_probe.py 64 > gpurun_out/tl_relaxed.log 2>&1 || { tail gpurun_out/tl_relaxed.log; exit 1; }
grep hpw gpurun_out/tl_strict.log gpurun_out/tl_relaxed.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py > gpurun_out/t4.log 2>&1 || { tail -20 gpurun_out/t4.log; exit 1; }
tail -1 gpurun_out/t4.log
timeout -k 10 600 python bench.py --workload c4 --steps 4 --warmup 2 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
