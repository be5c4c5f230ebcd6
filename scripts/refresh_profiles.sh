#!/bin/bash
# Everything profiles/r01 holds, from one GPU call: kernel-trace stats and the
# FETCH/WRITE byte passes (profile_round.sh), SQ counters, light phase stamps
# (timing build: make -C shadow-1_amd timing TIMING_FLAGS="-DSHD_TIMING_NOWAIT
# -DSHD_TIMING_LIGHT").  Outputs under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/profile_round.sh || exit 1
bash scripts/pmc_round.sh > gpurun_out/pmc_round.log 2>&1 || exit 2
python3 scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 --kernel k_round_tl > gpurun_out/sq_counters.txt || exit 3
SHD_TIMING_LIGHT=1 SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/round_timing.py --load 16 \
    > gpurun_out/round_timing.txt 2>&1 || exit 4
echo refresh done
