#!/bin/bash
# the sparse round's share gather polling 512 shares per round trip (W = 8) against 256: the
# sparse parity tests, then C5's shard, 250 k hosts and the one-rank group, two alternations
# (libshdgpu_w4.so: the same tree with W = 4)
set -o pipefail
O=gpurun_out/r05_gatherw
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -k sparse -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 2; }
tail -1 $O/tests.log
run() {  # tag lib extra
  local tag=$1 lib=$2; shift 2
  SHDGPU_LIB=$lib timeout -k 10 400 python3 bench.py --workload c5 --steps 2 --warmup 2 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])"
}
for rep in 1 2; do
  run w8_c5_$rep shadow-1_amd/libshdgpu.so --hosts-per-gpu 125000
  run w4_c5_$rep shadow-1_amd/libshdgpu_w4.so --hosts-per-gpu 125000
  run w8_h250_$rep shadow-1_amd/libshdgpu.so --hosts-per-gpu 250000
  run w4_h250_$rep shadow-1_amd/libshdgpu_w4.so --hosts-per-gpu 250000
done
