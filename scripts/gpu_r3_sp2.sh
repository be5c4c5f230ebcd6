#!/bin/bash
# round 3: k_round_sp after the record-load fix -- parity, phases, C5 shard bench
set -o pipefail
O=gpurun_out/r03/sp2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread -k "sparse or geometric_one" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -8
SHDGPU_LIB=shadow-1_amd/libshdgpu_tim.so timeout -k 10 300 python3 scripts/ps_timing.py --workload c5 --hosts 125000 > $O/sp_timing_c5.txt 2>&1 || { tail $O/sp_timing_c5.txt; exit 1; }
cat $O/sp_timing_c5.txt
timeout -k 10 400 python3 bench.py --no-cpu-baseline --lossy-edge-loss-max 0 --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 > $O/c5_125k.json 2> $O/c5_125k.err || { tail $O/c5_125k.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c5_125k.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c5_125k', round(d['value']/1e6,2), 'M', r['kernel'], r['avg_round_us'], 'us/round', r['packet_events_per_launch'], 'pkt/round')"
