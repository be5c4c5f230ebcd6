#!/bin/bash
# path-cache parity tests, then the APSP phase ablation
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pathcache_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tpc.log 2>&1 || { tail -40 gpurun_out/tpc.log; exit 1; }
tail -3 gpurun_out/tpc.log
bash scripts/apsp_phases.sh
