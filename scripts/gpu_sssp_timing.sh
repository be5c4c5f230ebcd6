#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pathcache_gpu.py > gpurun_out/tpc.log 2>&1 || { tail -20 gpurun_out/tpc.log; exit 1; }
tail -1 gpurun_out/tpc.log
SHDGPU_LIB=shadow-1_amd/libshdgpu_pcvt.so timeout -k 10 120 python -u scripts/sssp_timing.py 10000 > gpurun_out/sssp_timing.txt 2>&1 || { tail gpurun_out/sssp_timing.txt; exit 1; }
timeout -k 10 120 python -u scripts/apsp_timing.py > gpurun_out/apsp.json && grep -A3 geometric gpurun_out/apsp.json | head -4
cat gpurun_out/sssp_timing.txt
