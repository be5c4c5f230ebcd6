#!/bin/bash
# GPU suite, then the rate on the headline (hosts per wave 64) and the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/th.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/th.log | tail -15
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 scripts/hpw_probe.py 64 > gpurun_out/hpw_h.log 2>&1 || { tail gpurun_out/hpw_h.log; exit 2; }
grep hpw gpurun_out/hpw_h.log | cut -c1-400
timeout -k 10 300 python3 bench.py > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || { tail gpurun_out/bench_h.err; exit 3; }
cat gpurun_out/bench_h.json
