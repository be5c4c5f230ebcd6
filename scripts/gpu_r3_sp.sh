#!/bin/bash
# round 3: sparse persistent rounds (k_round_sp) -- parity, then the C5 shard / C4 / C3-100k benches
set -o pipefail
O=gpurun_out/r03/sp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread -k "sparse or geometric_one or bundled_complete" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -12
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; return 1; }
  python3 -c "
import json
d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$n', round(d['value']/1e6,2), 'M', r['kernel'], r['avg_round_us'], 'us/round', r['packet_events_per_launch'], 'pkt/round')"
}
run c5_125k --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 &&
run c4 --workload c4 --steps 2 --warmup 2 &&
run c3_100k --hosts-per-gpu 100000 --steps 2 --warmup 2
