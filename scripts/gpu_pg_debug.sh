#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/pg_debug.py > gpurun_out/pg_debug.txt 2>&1 || { tail -30 gpurun_out/pg_debug.txt; exit 1; }
cat gpurun_out/pg_debug.txt
