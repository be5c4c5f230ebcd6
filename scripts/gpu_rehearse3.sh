#!/bin/bash
# the multi-process group tests, then the bench's N > 1 path rehearsed with 2 and 3 ranks on one GPU
set -o pipefail
mkdir -p gpurun_out/reh
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_xgroup_procs_gpu.py > gpurun_out/tfuse.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tfuse.log | tail -5
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_rehearse.sh || exit 2
