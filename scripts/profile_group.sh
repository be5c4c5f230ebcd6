#!/bin/bash
# rocprofv3 kernel-trace summary of the engine-group bench at one rank (RCCL transport)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_group -o run -- \
    python3 bench.py --group --steps 2 --warmup 2 --no-cpu-baseline > gpurun_out/prof_group.json 2> gpurun_out/prof_group.err || exit 1
echo group profile done
