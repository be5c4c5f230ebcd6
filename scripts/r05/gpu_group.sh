#!/bin/bash
# round 5: the sparse fused group round (k_round_spx) -- group tests, then the
# C5 per-GPU shard through the one-rank group, k_round_px (SHD_X_NO_SP) against
# k_round_spx, alternated
set -o pipefail
O=gpurun_out/r05_group
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_xgroup_procs_gpu.py \
    tests/test_fullsize_gpu.py -k "sparse or multiprocess" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " $O/tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  SHD_X_NO_SP=1 timeout -k 10 400 python -u bench.py --workload c5 --hosts-per-gpu 125000 --group --steps 2 --warmup 2 \
      --no-cpu-baseline > $O/c5_px_$rep.json 2> $O/c5_px_$rep.err || exit 5
  timeout -k 10 400 python -u bench.py --workload c5 --hosts-per-gpu 125000 --group --steps 2 --warmup 2 \
      --no-cpu-baseline > $O/c5_spx_$rep.json 2> $O/c5_spx_$rep.err || exit 6
  python - <<PY
import json
for k in ("px", "spx"):
    d = json.load(open("$O/c5_%s_$rep.json" % k))
    r = d["roofline"]
    print(k, "rep $rep", round(d["value"] / 1e6, 2), "M pkt ev/s", r["kernel"], r["avg_round_us"], "us/round")
PY
done
