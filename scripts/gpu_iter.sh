#!/bin/bash
# one iteration: the GPU suite, the rate probe, the timed-region HBM bytes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/th.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/th.log | tail -15
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 scripts/hpw_probe.py 64 > gpurun_out/hpw_h.log 2>&1 || { tail gpurun_out/hpw_h.log; exit 2; }
grep hpw gpurun_out/hpw_h.log | cut -c1-300
./scripts/gpu_pmc_timed.sh > gpurun_out/pmc_timed.log 2>&1 || { tail gpurun_out/pmc_timed.log; exit 3; }
grep -E "timed|SIZE" gpurun_out/pmc_timed.log
