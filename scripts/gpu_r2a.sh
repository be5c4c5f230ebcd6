#!/bin/bash
# round 2: GPU tests, then the bench at two step/warm-up settings (reproducibility)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/b82.json 2> gpurun_out/b82.err || { tail gpurun_out/b82.err; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b205.json 2> gpurun_out/b205.err || { tail gpurun_out/b205.err; exit 1; }
cat gpurun_out/b82.json gpurun_out/b205.json
