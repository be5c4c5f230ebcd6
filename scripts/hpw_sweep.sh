set -e
mkdir -p gpurun_out
: > gpurun_out/sweep.log
for h in 64 32 16 8 4; do
  echo "== hpw $h" >> gpurun_out/sweep.log
  SHD_HPW=$h timeout -k 10 120 python scripts/prof_round.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/sweep.log
done
