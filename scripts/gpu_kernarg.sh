#!/bin/bash
# A/B: kernel arguments in device memory or not
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python3 scripts/hpw_probe.py 64 > gpurun_out/probe_ka$v.log 2>&1 || { tail gpurun_out/probe_ka$v.log; exit 2; }
  echo "HIP_FORCE_DEV_KERNARG=$v: $(grep hpw gpurun_out/probe_ka$v.log | cut -c1-60)"
done
