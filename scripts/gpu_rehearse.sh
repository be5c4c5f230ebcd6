#!/bin/bash
# the bench's N > 1 path on one GPU: 2 and 3 ranks over the host-memory communicator (gloo for torch.distributed)
set -o pipefail
mkdir -p gpurun_out/reh
for n in 2 3; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29530 + n)) bench.py --gpus $n --steps 3 --warmup 2 --no-cpu-baseline --comm host \
      > gpurun_out/reh/n$n.json 2> gpurun_out/reh/n$n.err || { tail -20 gpurun_out/reh/n$n.err; exit $n; }
  python3 -c "import json; d=json.load(open('gpurun_out/reh/n$n.json')); print($n, d['value'], d['ms_per_step'], d['rounds'], d['config']['exchange'], d['apsp']['sharded_build_ms'])"
done
