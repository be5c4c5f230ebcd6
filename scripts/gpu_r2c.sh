#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_model_gpu.py tests/test_boundary_gpu.py tests/test_xgroup_procs_gpu.py tests/test_fullsize_gpu.py \
    -k "not c5" > gpurun_out/t2.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t2.log | tail -40
[ $rc -le 1 ] || exit 1
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/b82c.json 2> gpurun_out/b82c.err || { tail gpurun_out/b82c.err; exit 1; }
cat gpurun_out/b82c.json
