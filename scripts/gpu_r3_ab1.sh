#!/bin/bash
# headline A/B: poll sleep in the persistent barrier (variant lib), then hosts per wave 32 / 48 (SHD_HPW)
set -o pipefail
O=gpurun_out/ab1
mkdir -p $O
: > $O/ab.log
run() {  # tag, env...
  local t=$1; shift
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline --lossy-edge-loss-max 0 --steps 4 > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$t.json')); print('$t', round(d['value']/1e6,2), d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])" | tee -a $O/ab.log
}
for k in 0 1; do
  run A$k X=1 && run S$k SHDGPU_LIB=shadow-1_amd/libshdgpu_var.so && run H32_$k SHD_HPW=32 && run H48_$k SHD_HPW=48 || exit 1
done
