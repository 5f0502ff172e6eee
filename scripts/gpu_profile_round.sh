# Round-end evidence: rocprof trace + PMC passes of the default bench, then the
# default bench line (with the CPU baseline) into gpurun_out/bench.json
set -o pipefail
TAG=${1:-r01}
bash scripts/profile.sh $TAG || exit 1
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.json | cut -c1-400
