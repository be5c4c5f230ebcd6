#!/bin/bash
# GPU tests, then the round-kernel timing sweep (plain and instrumented builds)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 120 python scripts/prof_round.py 2>&1 | grep -v amdgpu.ids
SHDGPU_LIB=shadow-1_amd/libshdgpu_prof.so timeout -k 10 120 python scripts/prof_round.py 2>&1 | grep -v amdgpu.ids
