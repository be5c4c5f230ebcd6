#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/t -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 > gpurun_out/gaps/b.json 2> gpurun_out/gaps/b.err || { tail gpurun_out/gaps/b.err; exit 1; }
python3 scripts/gap_stats.py gpurun_out/gaps/t > gpurun_out/gaps/stats.txt || exit 2
rm -rf gpurun_out/gaps/t
cat gpurun_out/gaps/stats.txt
