#!/bin/bash
# engine-group tests, then the single-rank RCCL group bench: ticketless rounds vs the ticketed k_round_x
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "group" > gpurun_out/tg.log 2>&1 || { tail -40 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
for v in tl ticket tl ticket; do
  if [ $v = ticket ]; then export SHD_X_TICKET=1; else unset SHD_X_TICKET; fi
  timeout -k 10 300 python -u bench.py --group --steps 3 --no-cpu-baseline > gpurun_out/bg_$v.json 2> gpurun_out/bg_$v.err || { tail -20 gpurun_out/bg_$v.err; exit 3; }
  python3 -c "import json;d=json.load(open('gpurun_out/bg_$v.json'));print('$v', d['value'], d['roofline']['avg_launch_us'], d['roofline']['avg_in_kernel_us'])"
done
