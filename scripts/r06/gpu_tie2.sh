#!/bin/bash
# round 6: k_sssp_tie_lds without workgroup barriers (a wave's own order; the parents' stores and the next
# pop's arc loads no longer drained twice a pop): parity, then the 10 k build times
set -o pipefail
O=gpurun_out/r06_tie2
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_pathcache_gpu.py \
    tests/test_pc_touches_gpu.py tests/test_ingress_gpu.py > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp.log 2>&1 && \
SHD_PC_TIE_HC=1536 timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_1536.log 2>&1
