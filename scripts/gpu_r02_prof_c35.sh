#!/bin/bash
# rocprofv3 trace + 4 PMC passes of the C3 and C5 bench runs (profiles/r02_c3, r02_c5)
set -o pipefail
bash scripts/profile.sh r02_c3 --config C3 --steps 20 || exit 1
bash scripts/profile.sh r02_c5 --config C5 --steps 2 --warmup 1 || exit 1
