#!/bin/bash
# MFMA backward pass: the -m gpu suite on the tree's library, then same-box A/B of
# the backward kernel (fb_bwd4_kernel variants vs fb_bwd2_kernel, VBHEM_NO_BWD4=1).
#   scripts/gpu_bwd4.sh TAG [variant.so ...]
set -o pipefail
TAG=${1:-bwd4}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
[ "$NOTEST" = 1 ] || timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; [ "$NOTEST" = 1 ] || tail -3 $OUT/tests.log; [ "$NOTEST" != 1 ] && [ $rc -ne 0 ] && exit $rc
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-parity-sample --no-shard-sim --em-iters 0"
one() {  # label, then env assignments
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py $ARGS > $OUT/ab_$lab.json 2>$OUT/ab_$lab.err || return 1
  tail -1 $OUT/ab_$lab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lab', 'ms',round(d['ms_per_step'],4),'bwd',round(d['roofline']['kernel_ms'],4),'fwd',round(d['gated_forward']['kernel_ms'],4),'stats',round(d['stats_kernels_ms_per_step'],4))"
}
for rep in 1 2; do
  one tree_$rep VBHEM_X=1 || exit 1
  one nolist4_$rep VBHEM_NO_LIST4=1 || exit 1
  one bwd2_$rep VBHEM_NO_BWD4=1 VBHEM_NO_LIST4=1 || exit 1
  for lib in "$@"; do one $(basename $lib .so)_$rep VBHEM_LIB_PATH=$(realpath $lib) || exit 1; done
done
# PMC passes (the tree's library) when PMC=1: instruction mix and waits of the C4 step
if [ "$PMC" = 1 ]; then
  bash scripts/pmc.sh $TAG "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
    "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS" \
    -- --steps 3 --warmup 1 --no-parity-sample --no-shard-sim --em-iters 0 || exit 1
fi
