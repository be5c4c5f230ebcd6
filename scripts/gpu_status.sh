#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/ts.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/ts.log | tail -8
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/ts.log | head -80; exit 1; }
timeout -k 10 300 python3 scripts/hpw_probe.py 64 > gpurun_out/probe.log 2>&1 && grep hpw gpurun_out/probe.log | cut -c1-120
