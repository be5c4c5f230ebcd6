#!/bin/bash
# rocprofv3 kernel-trace summary + per-dispatch HBM byte counters for the bench
# workload (run on the GPU box from the repo root; outputs under gpurun_out/prof_*)
set -o pipefail
export TMPDIR=/tmp
STEPS=${STEPS:-2}
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- \
    python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- \
    python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 > /dev/null 2> gpurun_out/prof_fetch.err || exit 2
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- \
    python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 > /dev/null 2> gpurun_out/prof_write.err || exit 3
python3 scripts/pmc_bytes.py gpurun_out/prof_fetch gpurun_out/prof_write --out gpurun_out/k_round_pmc_bytes.json > /dev/null || exit 4
echo profile done
