#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/diag_active.py 480 2 240 &&
SHD_NO_TL=1 timeout -k 10 120 python3 scripts/diag_active.py 480 2 240 &&
timeout -k 10 200 python3 scripts/diag_active.py 20000 2 &&
SHD_NO_TL=1 timeout -k 10 200 python3 scripts/diag_active.py 20000 2
