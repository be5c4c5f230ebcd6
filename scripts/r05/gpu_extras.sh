#!/bin/bash
# round 5: the other workloads' lines on the final tree -- the TCP bench under
# rocprofv3 --kernel-trace --stats, the C5 shard (single engine, sparse
# persistent) and the Tor-scale C4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_extras
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- \
    python3 bench.py --workload tcp --no-cpu-baseline --steps 2 --warmup 1 > $O/tcp_bench.json 2> $O/tr.err || { tail -5 $O/tr.err; exit 2; }
cp "$(find $O/tr -name '*kernel_stats.csv' | head -1)" $O/tcp_kernel_stats.csv && rm -rf $O/tr || exit 3
head -4 $O/tcp_kernel_stats.csv; tail -1 $O/tcp_bench.json | cut -c1-300
timeout -k 10 500 python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline \
    > $O/c5_shard.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 4; }
timeout -k 10 500 python3 bench.py --workload c4 --steps 2 --warmup 2 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 5; }
python3 - <<PY
import json
for k in ("c5_shard", "c4"):
    d = json.load(open("$O/%s.json" % k)); r = d["roofline"]
    print(k, round(d["value"] / 1e6, 2), "M", r["kernel"], r.get("avg_round_us"), "us/round")
PY
