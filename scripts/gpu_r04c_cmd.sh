# GPU suite (incl. the new S = 12 MFMA backward), stats ring-depth A/B at C4 and at the
# 12,500-base shard, C5 A/B of the backward kernels (bwd12 3 / 2 waves vs fb_bwd2_kernel),
# then C3 / C5 bench lines
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
# ordinary test failures (rc 1) do not stop the measurements; a crash, abort or time
# limit does
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 bash scripts/ab_lib.sh build/ab/pd3.so build/ab/pd4.so build/ab/q2w2.so build/ab/q2w3.so build/ab/ru2.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
timeout -k 10 600 bash scripts/ab_lib.sh --args "--steps 20 --warmup 3 --N 12500" build/ab/pd3.so build/ab/pd4.so build/ab/ru2.so > $OUT/ab_12k.txt 2>&1; cat $OUT/ab_12k.txt
C5ARGS="--config C5 --steps 4 --warmup 1 --no-cpu-baseline --no-shard-sim --em-iters 0 --parity-seconds 3"
for v in tree b12w2 bwd2; do
  case $v in tree) E="";; b12w2) E="VBHEM_LIB_PATH=$(realpath build/ab/b12w2.so)";; bwd2) E="VBHEM_NO_BWD12=1";; esac
  env $E timeout -k 10 400 python -u bench.py $C5ARGS > $OUT/c5_$v.json 2> $OUT/c5_$v.err || exit 1
  tail -1 $OUT/c5_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); ps=d.get('parity_sample') or {}; print('$v', 'ms',round(d['ms_per_step'],3),'bwd',round(d['roofline']['kernel_ms'],4), d['roofline']['kernel'], 'em',round(d['emission_kernel_ms'],4),'fwd',round(d['gated_forward']['kernel_ms'],4),'stats',round(d['stats_kernels_ms_per_step'],3),'LLerr',ps.get('LL_elbo_max_rel_err'),'hz',ps.get('hat_Z_max_err'))"
done
for cfg in C3 C5; do
  timeout -k 10 500 python -u bench.py --config $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err || exit 1
  tail -c 300 $OUT/bench_$cfg.json; echo
done
