#!/bin/bash
# the headline rate only, for A/B runs of the round kernel: hosts per wave as arguments (default 64)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 scripts/hpw_probe.py "$@" > gpurun_out/probe.log 2>&1 || { tail gpurun_out/probe.log; exit 2; }
grep hpw gpurun_out/probe.log | cut -c1-400
