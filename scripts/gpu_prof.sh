#!/bin/bash
# per-phase timing of the round kernel (plain + instrumented), then rocprofv3 kernel-trace summary of bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python scripts/prof_round.py > gpurun_out/prof_plain.txt 2>&1 || { tail gpurun_out/prof_plain.txt; exit 1; }
SHDGPU_LIB=shadow-1_amd/libshdgpu_prof.so timeout -k 10 180 python scripts/prof_round.py > gpurun_out/prof_inst.txt 2>&1 || { tail gpurun_out/prof_inst.txt; exit 2; }
grep -v amdgpu.ids gpurun_out/prof_plain.txt gpurun_out/prof_inst.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- \
    python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit 3
cat gpurun_out/prof_bench.json
find gpurun_out/prof_trace -name "*stats*"
