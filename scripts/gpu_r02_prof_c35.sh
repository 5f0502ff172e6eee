#!/bin/bash
# rocprofv3 trace + 4 PMC passes of the C3 and C5 bench runs (profiles/TAG_c3, TAG_c5)
TAG=${1:-r02}
set -o pipefail
bash scripts/profile.sh ${TAG}_c3 --config C3 --steps 20 || exit 1
bash scripts/profile.sh ${TAG}_c5 --config C5 --steps 2 --warmup 1 || exit 1
