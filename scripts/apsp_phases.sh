#!/bin/bash
# APSP phase ablation: full build vs Bellman-Ford only (pcv1) vs + parents (pcv2).
# Build first: make -C shadow-1_amd pcvariant PC_FLAGS=-DSHD_SSSP_STOP_AFTER=1 PCV=1 (and 2).
set -o pipefail
mkdir -p gpurun_out
for lib in libshdgpu.so libshdgpu_pcv1.so libshdgpu_pcv2.so ${EXTRA_LIBS}; do
  echo "== $lib"
  SHDGPU_LIB=shadow-1_amd/$lib timeout -k 10 120 python -u scripts/apsp_timing.py > gpurun_out/apsp_$lib.json 2> gpurun_out/apsp_$lib.err || { tail gpurun_out/apsp_$lib.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/apsp_$lib.json'));print({k:(v['ms'],v.get('sssp_ms')) for k,v in d.items()})"
done
