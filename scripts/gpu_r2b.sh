#!/bin/bash
# round 2: the new GPU tests (model features, full-size fixtures, boundary adapters,
# multi-process group), then the bench with its CPU baseline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_model_gpu.py tests/test_boundary_gpu.py tests/test_xgroup_procs_gpu.py tests/test_fullsize_gpu.py \
    -k "not c5" > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/b82c.json 2> gpurun_out/b82c.err || { tail gpurun_out/b82c.err; exit 1; }
cat gpurun_out/b82c.json
