#!/bin/bash
# round 3, session 2: path cache (batched frontier loads), the engine against
# the reference loop's fixtures, the group tests (timeout / region fallback),
# the per-GPU shards with the density-chosen batches
set -o pipefail
O=gpurun_out/r03s2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_pathcache_gpu.py tests/test_ref_loop_gpu.py tests/test_xgroup_procs_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log
timeout -k 10 120 python -u scripts/apsp_timing.py > $O/apsp.json 2> $O/apsp.err || { tail $O/apsp.err; exit 2; }
python3 -c "import json;d=json.load(open('$O/apsp.json'));print({k:(round(v['ms'],3),round(v.get('sssp_ms'),3)) for k,v in d.items()})"
HOSTS_OUT=$O/hosts bash scripts/gpu_r3_hosts.sh || exit 3
