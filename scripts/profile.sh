#!/bin/bash
# Profile bench.py on the GPU box: kernel trace + stats, then separate PMC passes.
# Usage: scripts/profile.sh TAG [bench args...]   (PASSES=trace: the kernel trace only)
set -o pipefail
TAG=${1:-run}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$@"
# the PMC passes run the full-size E-steps only (no shard simulation, no EM-loop
# timing): every launch of a kernel then has the same size and the per-dispatch
# averages are the full-size launch's counters (prof_summary.py records this)
PMC_ARGS="--no-shard-sim --em-iters 0 --no-parity-sample --steps 6 --warmup 2 --settle-ms 0"
run() {  # name, extra rocprof args
  local name=$1; shift
  local extra=$ARGS
  case $name in pmc*) extra="$ARGS $PMC_ARGS";; trace) extra="$ARGS $TRACE_ARGS";; esac
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline $extra > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
# the traced run skips the shard simulation too, so every launch of a kernel in the
# trace is the same size and the trace's mean launch time reproduces the bench's
# roofline (prof_summary.py roofline_check); profile the shard size as its own
# command (scripts/profile.sh TAG_shard --N 12500)
TRACE_ARGS="--no-shard-sim"
echo "$ARGS $TRACE_ARGS" > $OUT/trace_args.txt
echo "$PMC_ARGS" > $OUT/pmc_args.txt
run trace --kernel-trace --stats || exit $?
[ "$PASSES" = trace ] && exit 0
run pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run pmc2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAIT_INST_LDS &&
run pmc3 --pmc FETCH_SIZE &&
run pmc4 --pmc WRITE_SIZE &&
run pmc5 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
