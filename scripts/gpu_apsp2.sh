#!/bin/bash
# path-cache changes: the path-cache GPU tests, then the APSP build times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pathcache_gpu.py tests/test_boundary_gpu.py > gpurun_out/tpc.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tpc.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u scripts/apsp_timing.py > gpurun_out/apsp.json 2> gpurun_out/apsp.err || { tail gpurun_out/apsp.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/apsp.json'));print({k:(round(v['ms'],3),round(v.get('sssp_ms'),3)) for k,v in d.items()})"
