#!/bin/bash
# kernel traces: the 12,500-base C4 shard (bench --N 12500) and C3
set -o pipefail
PASSES=trace bash scripts/profile.sh s12 --N 12500 --steps 40 --warmup 5 --no-shard-sim --em-iters 0 --no-parity-sample || exit $?
PASSES=trace bash scripts/profile.sh c3 --config C3 --steps 40 --warmup 5 --no-shard-sim --em-iters 0 --no-parity-sample
