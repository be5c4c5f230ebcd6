#!/bin/bash
set -o pipefail
bash scripts/r06/gpu_grouplean.sh && bash scripts/r06/gpu_tiehc.sh
