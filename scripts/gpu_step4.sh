#!/bin/bash
# C5 emission variants: bitwise vs VBHEM_EM_NODB, and timing.  scripts/gpu_step4.sh TAG lib...
set -o pipefail
TAG=${1:-r06g}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
VBHEM_EM_NODB=1 timeout -k 10 300 python scripts/cmp_libs.py dump $OUT/nodb.npz > $OUT/cmp.txt 2>&1 || { tail $OUT/cmp.txt; exit 1; }
for lib in "$@"; do
  n=$(basename $lib .so)
  VBHEM_LIB_PATH=$(pwd)/$lib timeout -k 10 300 python scripts/cmp_libs.py dump $OUT/$n.npz >> $OUT/cmp.txt 2>&1 || { tail $OUT/cmp.txt; exit 1; }
  echo "== $n vs nodb"; python scripts/cmp_libs.py diff $OUT/$n.npz $OUT/nodb.npz | tee -a $OUT/cmp.txt | grep C5
done
bash scripts/ab_lib.sh --args "--config C5 --steps 3 --warmup 1" "$@" > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt
VBHEM_EM_NODB=1 timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $OUT/nodb_c5.json 2>&1; tail -1 $OUT/nodb_c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nodb ms', d['ms_per_step'], 'em', d['emission_kernel_ms'])"
