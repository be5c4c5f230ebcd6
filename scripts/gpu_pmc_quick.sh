#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per k_round_tl dispatch (two passes) on the headline -> gpurun_out/pmcq/k_round_pmc_bytes.json
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmcq
rm -rf $O; mkdir -p $O
ARGS="--steps 2 --warmup 2 --no-cpu-baseline --lossy-edge-loss-max 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
    python3 bench.py $ARGS > $O/fetch_bench.json 2> $O/fetch.err || { tail $O/fetch.err; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
    python3 bench.py $ARGS > $O/write_bench.json 2> $O/write.err || { tail $O/write.err; exit 4; }
python3 scripts/pmc_bytes.py $O/fetch $O/write --fetch-bench $O/fetch_bench.json --write-bench $O/write_bench.json \
    --out $O/k_round_pmc_bytes.json && rm -rf $O/fetch $O/write || exit 5
cat $O/k_round_pmc_bytes.json
