#!/bin/bash
# the whole GPU suite, then per-event-class cycle costs (timing build, full stamps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/tall.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tall.log | tail -15
[ $rc -eq 0 ] || exit 1
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 200 python3 scripts/round_timing.py --load 16 \
    > gpurun_out/round_timing_full.txt 2>&1 || { tail gpurun_out/round_timing_full.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/round_timing_full.txt
bash scripts/profile_round.sh || exit 2
bash scripts/pmc_round.sh > gpurun_out/pmc_round.log 2>&1 || exit 3
python3 scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 --kernel k_round_tl > gpurun_out/sq_counters.txt || exit 4
cat gpurun_out/k_round_pmc_bytes.json
