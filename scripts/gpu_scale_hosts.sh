#!/bin/bash
# hosts per GPU: the C3-shaped lossless PHOLD at 100 k and 1 M hosts on one GPU, and BASELINE C5 (1 M hosts, CoDel, loss) on one GPU
set -o pipefail
mkdir -p gpurun_out/hosts
O=gpurun_out/hosts
timeout -k 10 300 python3 bench.py --hosts-per-gpu 100000 --steps 2 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 \
    > $O/c3_100k.json 2> $O/c3_100k.err || { tail $O/c3_100k.err; exit 1; }
timeout -k 10 400 python3 bench.py --hosts-per-gpu 1000000 --steps 2 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0 \
    > $O/c3_1m.json 2> $O/c3_1m.err || { tail $O/c3_1m.err; exit 2; }
timeout -k 10 400 python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline \
    > $O/c5_1m.json 2> $O/c5_1m.err || { tail $O/c5_1m.err; exit 3; }
for f in c3_100k c3_1m c5_1m; do
python3 -c "import json; d=json.load(open('$O/$f.json')); r=d['roofline']; print('$f', d['config']['hosts'], round(d['value']/1e6,1), 'M/s', d['ms_per_step'], 'ms/step', d['rounds'], 'rounds', r['avg_launch_us'], 'us/launch', r['packet_events_per_launch'])"
done
