# A/B: fallback scratch last in the workspace (tree) vs the previous commit (head), the
# same code with the scratch first (cur), resp_kernel at 3 waves per SIMD (wpe3);
# C4 without the fold; C3; kernel trace of a 12,500-base C4 shard
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
timeout -k 10 900 bash scripts/ab_lib.sh build/ab/head.so build/ab/cur.so build/ab/wpe3.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
VBHEM_NO_FOLD_EXACT=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $OUT/nofold.json 2>&1 && tail -1 $OUT/nofold.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nofold ms', round(d['ms_per_step'],4), 'stats', round(d['stats_kernels_ms_per_step'],4))"
timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/head.so build/ab/wpe3.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr12k -o tr12k --output-format csv -- python3 bench.py --N 12500 --steps 20 --warmup 3 --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $OUT/tr12k.log 2>&1
f=$(find $OUT/tr12k -name "*kernel_trace.csv" | head -1); d=$(dirname $f); cp $f $d/run_kernel_trace.csv && python3 scripts/trace_gaps.py $d > $OUT/gaps12k.txt; cat $OUT/gaps12k.txt
