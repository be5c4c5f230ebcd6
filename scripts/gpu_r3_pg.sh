#!/bin/bash
# round 3 final: the whole GPU suite, the one-rank group A/B (SHD_X_PG=1: the opt-in persistent
# group batches, against the default fused schedule) and the single engine, the per-GPU shards
set -o pipefail
O=gpurun_out/pg
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag, env..., -- args
  local t=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --lossy-edge-loss-max 0 --steps 4 $BARGS > $O/$t.json 2> $O/$t.err || { tail -5 $O/$t.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$t.json')); r=d['roofline']; print('$t', round(d['value']/1e6,2), r['kernel'], r['avg_round_us'], d['config'].get('exchange'))"
}
BARGS="--group --exchange p2p" run pg SHD_X_PG=1 && BARGS="--group --exchange p2p" run px X=1 && run single X=1
HOSTS_OUT=$O/hosts bash scripts/gpu_r3_hosts.sh || exit 3
