#!/bin/bash
# round 6, final engine: the C4 Tor-scale line and C3 at 100 k hosts, with the warm-up (2 steps) the earlier
# round-6 measurements used (1 step leaves the lazy path cache's warm-up in the timed window)
set -o pipefail
O=gpurun_out/r06_c4
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 bench.py --workload c4 --no-cpu-baseline --lossy-edge-loss-max 0 --steps 2 --warmup 2 \
    > $O/c4.json 2> $O/c4.err || exit 3
timeout -k 10 400 python3 bench.py --hosts-per-gpu 100000 --no-cpu-baseline --lossy-edge-loss-max 0 --steps 2 --warmup 2 \
    > $O/c3_100k.json 2> $O/c3_100k.err || exit 4
rm -f $O/*.err
