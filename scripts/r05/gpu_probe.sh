#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05_probe
timeout -k 10 300 python -u scripts/r05/tcp_wide_probe.py 2>&1 | tee gpurun_out/r05_probe/wide.log
