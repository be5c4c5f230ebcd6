#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash scripts/apsp_phases.sh || exit 1
CFGS="20000 10000|40000 10000|80000 10000" 
IFS='|'; for cfg in $CFGS; do IFS=' '; set -- $cfg
  echo "hosts=$1"
  timeout -k 10 200 python -u bench.py --hosts-per-gpu $1 --vertices $2 --steps 1 --warmup 2 --no-cpu-baseline > gpurun_out/scale_$1_$2.json 2> gpurun_out/scale_$1_$2.err
  echo "rc=$?"; tail -c 300 gpurun_out/scale_$1_$2.err; python3 -c "import json;d=json.load(open('gpurun_out/scale_$1_$2.json'));print(d['value'])" || true
done
