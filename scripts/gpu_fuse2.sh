#!/bin/bash
# fused peer-to-peer rounds: the multi-process group tests, then the one-rank group rate: header replicas 8 / 1, unfused
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_xgroup_procs_gpu.py > gpurun_out/tfuse.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tfuse.log | tail -5
[ $rc -eq 0 ] || exit 1
ARGS="--group --exchange p2p --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/gfused.json 2> gpurun_out/gfused.err || { tail gpurun_out/gfused.err; exit 2; }
SHD_X_REPL=1 timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/grep1.json 2> gpurun_out/grep1.err || { tail gpurun_out/grep1.err; exit 3; }
SHD_X_UNFUSED=1 timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/gunfused.json 2> gpurun_out/gunfused.err || { tail gpurun_out/gunfused.err; exit 4; }
for f in gfused grep1 gunfused; do
python3 -c "import json,sys; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['rounds'])"
done
