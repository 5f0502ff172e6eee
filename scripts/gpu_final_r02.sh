#!/bin/bash
# Round-end evidence in one call: C4 kernel trace + 4 PMC passes + the default
# bench line (with the CPU baseline), the strong-scaling shard sizes, C3 and C5
# bench lines.  TAG names profiles/TAG_*.
set -o pipefail
TAG=${1:-r02f}
mkdir -p gpurun_out
bash scripts/gpu_profile_round.sh ${TAG}_c4 || exit 1
cp gpurun_out/bench.json gpurun_out/${TAG}_c4_bench.json
bash scripts/strong_sim.sh > gpurun_out/${TAG}_strong.txt 2>&1 || { cat gpurun_out/${TAG}_strong.txt; exit 1; }
cat gpurun_out/${TAG}_strong.txt
timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/c3.err || { tail gpurun_out/c3.err; exit 1; }
timeout -k 10 400 python bench.py --config C5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/c5.err || { tail gpurun_out/c5.err; exit 1; }
for c in c3 c5; do tail -1 gpurun_out/${TAG}_${c}_bench.json | cut -c1-260; done
