# K1 inside fb_bwd4_kernel / fb_list4_kernel (no emission GEMM, no E buffer at C4):
# the S = 8 parity tests, A/B against the previous commit's library (head) and the
# same tree with VBHEM_NO_K1_FUSE=1, per-kernel traces of both libraries at C4
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "S8 or C4 or c4 or gated or fused or list4 or mfma or fallback or exact or bwd4" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
PARITY=1 timeout -k 10 900 bash scripts/ab_lib.sh build/ab/head.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
VBHEM_NO_K1_FUSE=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $OUT/nok1.json 2>&1 && tail -1 $OUT/nok1.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nok1 ms', round(d['ms_per_step'],4), 'bwd', round(d['roofline']['kernel_ms'],4), 'stats', round(d['stats_kernels_ms_per_step'],4))"
for lib in tree head; do
  if [ $lib = head ]; then export VBHEM_LIB_PATH=$(realpath build/ab/head.so); else unset VBHEM_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_$lib -o tr --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $OUT/tr_$lib.log 2>&1
  f=$(find $OUT/tr_$lib -name "*kernel_stats.csv" | head -1); echo "== $lib"; cut -d, -f1-5 $f | head -14
done
unset VBHEM_LIB_PATH
