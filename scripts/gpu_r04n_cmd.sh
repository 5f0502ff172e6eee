# timelines (kernel trace gaps) of the C3 step and the 12,500-base C4 shard step
set -o pipefail
OUT=gpurun_out/r04n; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in C3 C4; do
  extra=""; [ $c = C4 ] && extra="--N 12500"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tr_$c -o tr --output-format csv -- python3 $R/bench.py --config $c $extra --steps 40 --warmup 5 --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $R/$OUT/tr_$c.log 2>&1 || exit 1
  f=$(find $R/$OUT/tr_$c -name "*kernel_trace.csv" | head -1); d=$(dirname $f); cp $f $d/run_kernel_trace.csv
  python3 $R/scripts/trace_gaps.py $d > $R/$OUT/gaps_$c.txt; cat $R/$OUT/gaps_$c.txt
done
