set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 60 ./scripts/microbench/launch > gpurun_out/r03/launch.txt 2>&1 || { cat gpurun_out/r03/launch.txt; exit 1; }
timeout -k 10 60 ./scripts/microbench/barrier > gpurun_out/r03/barrier.txt 2>&1 || { cat gpurun_out/r03/barrier.txt; exit 2; }
cat gpurun_out/r03/launch.txt gpurun_out/r03/barrier.txt
timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/r03/bench0.json 2> gpurun_out/r03/bench0.err || { tail gpurun_out/r03/bench0.err; exit 3; }
cat gpurun_out/r03/bench0.json | head -c 600
