#!/bin/bash
# round 3: shared deferred-send pool -- parity suite, then C4 / C3 / C5-shard benches
set -o pipefail
O=gpurun_out/r03/pool
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_model_gpu.py tests/test_ingress_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python3 -c "
import json
d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$n', round(d['value']/1e6,2), 'M', r['kernel'], r['avg_round_us'], 'us/round', r['packet_events_per_launch'], 'pkt/round')"
}
run c4 --workload c4 --steps 2 --warmup 2 &&
run c3 --steps 4 --warmup 2 &&
run c5_125k --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2
