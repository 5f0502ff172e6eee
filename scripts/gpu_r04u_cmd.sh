# stats_list_m_kernel block count at the 12,500-base shard and at C4 (VBHEM_SU_BLOCKS)
set -o pipefail
OUT=gpurun_out/r04u; mkdir -p $OUT
for rep in 1 2; do
for a in "--N 12500 --steps 40 --warmup 5" "--steps 20 --warmup 3"; do
  for nb in default 256 512 1024 1536; do
    if [ $nb = default ]; then unset VBHEM_SU_BLOCKS; else export VBHEM_SU_BLOCKS=$nb; fi
    timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $OUT/b.json 2>&1 || { tail -5 $OUT/b.json; exit 1; }
    tail -1 $OUT/b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a'.split('--steps')[0] or 'C4', 'blocks=$nb', 'ms', round(d['ms_per_step'],4), 'stats', round(d['stats_kernels_ms_per_step'],4))"
  done
done
done
unset VBHEM_SU_BLOCKS
