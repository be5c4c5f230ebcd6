#!/bin/bash
# round 3 final build: GPU suite, bench line, per-GPU shards, then profiles/r03 refresh
set -o pipefail
bash scripts/gpu_r3_check.sh && bash scripts/refresh_r03.sh
