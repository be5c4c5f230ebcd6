#!/bin/bash
# engine-group changes: the group tests (in-process groups, multi-process both transports), then the one-rank group rate
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_xgroup_procs_gpu.py tests/test_engine_gpu.py tests/test_model_gpu.py > gpurun_out/tg.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/tg.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 bench.py --group --exchange p2p --steps 4 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 \
    > gpurun_out/group_p2p.json 2> gpurun_out/group_p2p.err || { tail gpurun_out/group_p2p.err; exit 2; }
python3 -c "import json; d=json.load(open('gpurun_out/group_p2p.json')); print('p2p group', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])"
