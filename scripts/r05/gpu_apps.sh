#!/bin/bash
# round 5: the general datagram application (SHD_APP_UDP) -- reference-loop
# fixtures, the oracle at scale, refused models; engine regressions; C3 bench
set -o pipefail
O=gpurun_out/r05_apps
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_ref_loop_gpu.py \
    tests/test_app_gpu.py tests/test_engine_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-reference-cpu > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"; python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print(round(d['value']/1e6,2), 'M pkt ev/s', r['kernel'], r.get('avg_round_us'))"
