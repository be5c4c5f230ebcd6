set -e
mkdir -p gpurun_out
: > gpurun_out/load_sweep.log
for ld in 1 4 16 64; do
  echo "== load $ld" >> gpurun_out/load_sweep.log
  timeout -k 10 120 python scripts/prof_round.py --load $ld 2>&1 | grep -v amdgpu.ids >> gpurun_out/load_sweep.log
done
for h in 2000 40000; do
  echo "== hosts $h" >> gpurun_out/load_sweep.log
  timeout -k 10 120 python scripts/prof_round.py --hosts $h --vertices $h 2>&1 | grep -v amdgpu.ids >> gpurun_out/load_sweep.log
done
