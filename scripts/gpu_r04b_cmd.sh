# stats ring-depth A/B at C4 and at the 12,500-base shard, then C3 / C5 bench lines
set -o pipefail
mkdir -p gpurun_out/r04b
timeout -k 10 600 bash scripts/ab_lib.sh build/ab/pd3.so build/ab/pd4.so > gpurun_out/r04b/ab_c4.txt 2>&1; cat gpurun_out/r04b/ab_c4.txt
timeout -k 10 600 bash scripts/ab_lib.sh --args "--steps 20 --warmup 3 --N 12500" build/ab/pd3.so build/ab/pd4.so > gpurun_out/r04b/ab_12k.txt 2>&1; cat gpurun_out/r04b/ab_12k.txt
for cfg in C3 C5; do
  timeout -k 10 500 python -u bench.py --config $cfg > gpurun_out/r04b/bench_$cfg.json 2> gpurun_out/r04b/bench_$cfg.err || exit 1
  tail -c 300 gpurun_out/r04b/bench_$cfg.json; echo
done
