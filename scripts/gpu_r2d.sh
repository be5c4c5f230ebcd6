#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_model_gpu.py > gpurun_out/t3.log 2>&1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/t3.log | tail -10
timeout -k 10 300 python -u scripts/hpw_probe.py 64 32 16 > gpurun_out/hpw.log 2>&1 || { tail gpurun_out/hpw.log; exit 1; }
cat gpurun_out/hpw.log | grep -v amdgpu.ids
timeout -k 10 500 python bench.py --workload c4 --steps 4 --warmup 2 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail gpurun_out/c4.err; exit 1; }
cat gpurun_out/c4.json
