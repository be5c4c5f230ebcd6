#!/bin/bash
# round 6: the sparse round at the C5 shard -- A/B of the barrier's poll width (8 shares per lane per
# poll against 4) and of the block size (sph 256 default, 128, 192), two alternations; then the SQ
# counters of k_round_sp (two --pmc passes of the same bench command)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_sp3
mkdir -p $O
B="python3 bench.py --workload c5 --hosts-per-gpu 125000 --steps 2 --warmup 2 --no-cpu-baseline"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 $B > $O/$tag.json 2> $O/$tag.err || exit 3
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'])" >> $O/summary.txt
}
for rep in 1 2; do
  run def_$rep X=1
  run g4_$rep SHDGPU_LIB=shadow-1_amd/libshdgpu_var_g4.so
  run s128_$rep SHD_SP_HOSTS=128
  run s192_$rep SHD_SP_HOSTS=192
done
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" ; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/pmc$i -o run -- python3 bench.py --workload c5 \
      --hosts-per-gpu 125000 --steps 1 --warmup 2 --no-cpu-baseline > $O/pmc$i.out 2> $O/pmc$i.err || { tail -5 $O/pmc$i.err; exit 8; }
done
python3 scripts/pmc_summary.py $O/pmc1 $O/pmc2 --kernel k_round_sp > $O/sq_counters.txt && rm -rf $O/pmc1 $O/pmc2
