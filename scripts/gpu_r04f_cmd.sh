# wave-parallel exact fallback: the fallback tests, then the adversarial case at full
# size (C4, N = 100,000: every base's cluster-0 pair flagged twice), folded vs separate
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "fallback or exact" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python -u scripts/fold_bench.py 100000 > $OUT/fold.json 2> $OUT/fold.err || { tail -20 $OUT/fold.err; exit 1; }
cat $OUT/fold.json
