#!/bin/bash
# engine-group tests, then the single-rank RCCL group bench (graph-captured batches) and without graphs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "group" > gpurun_out/tg.log 2>&1 || { tail -40 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
timeout -k 10 300 python -u bench.py --group --steps 3 --no-cpu-baseline > gpurun_out/bench_group.json 2> gpurun_out/bench_group.err || { tail -20 gpurun_out/bench_group.err; exit 3; }
grep -v "amdgpu.ids\|RCCL\|HIP version\|ROCm version\|Hostname\|Librccl" gpurun_out/bench_group.err | tail -3
python3 -c "import json;d=json.loads(open('gpurun_out/bench_group.json').read().strip().splitlines()[-1]);print('graph', d['value'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])"
SHD_NO_GRAPH=1 timeout -k 10 300 python -u bench.py --group --steps 3 --no-cpu-baseline > gpurun_out/bench_group_ng.json 2> gpurun_out/bench_group_ng.err || { tail -20 gpurun_out/bench_group_ng.err; exit 4; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_group_ng.json'));print('nograph', d['value'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])"
