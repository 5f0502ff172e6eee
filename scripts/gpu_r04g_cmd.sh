# wave-parallel exact fallback, round 2 (inputs staged in LDS, resp_kernel capped at
# 4 waves per SIMD): fallback tests, A/B against the previous commit's library at C4
# and C3, the adversarial case at full size
set -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "fallback or exact" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 900 bash scripts/ab_lib.sh build/ab/head.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/head.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt
timeout -k 10 600 python -u scripts/fold_bench.py 100000 > $OUT/fold.json 2> $OUT/fold.err || { tail -20 $OUT/fold.err; exit 1; }
cat $OUT/fold.json
