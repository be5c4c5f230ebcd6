#!/bin/bash
# round 6: tied rows on k_sssp_tie_lds (one row per wave, heap in LDS): path-cache parity (the lane-heap
# kernel forced too, and a heap past LDS falling back), then the 10 k build times (tie-free / whole-ms)
set -o pipefail
O=gpurun_out/r06_tie
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_pathcache_gpu.py \
    tests/test_pc_touches_gpu.py tests/test_ingress_gpu.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/r05/apsp_ties.py > $O/apsp.log 2>&1 && \
SHD_PC_TIE_GLOBAL=1 timeout -k 10 300 python3 -u scripts/r05/apsp_ties.py > $O/apsp_global.log 2>&1
