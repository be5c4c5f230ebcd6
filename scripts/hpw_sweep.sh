set -e
for h in 64 16 8 4 2 1; do
  echo "== hpw $h" >> gpurun_out/sweep.log
  SHD_HPW=$h timeout -k 10 120 python scripts/prof_round.py >> gpurun_out/sweep.log 2>&1
  SHD_HPW=$h SHDGPU_LIB=shadow-1_amd/libshdgpu_prof.so timeout -k 10 120 python scripts/prof_round.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/sweep.log || true
done
