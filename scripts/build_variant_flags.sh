#!/bin/bash
# A library variant where ONE source gets extra compiler flags (e.g. an LLVM scheduling
# strategy):  scripts/build_variant_flags.sh OUT.so SOURCE.hip "FLAGS..."
set -e
OUT=$1; ONE=$2; EXTRA=$3
PKG=clustering-hidden-markov-models-with-variational-bayesian-hierarchical-em_amd
TMP=$(mktemp -d); objs=()
for src in $PKG/csrc/*.hip; do
  f=$(basename $src); fl=""
  [ "$f" = "$(basename $ONE)" ] && fl="$EXTRA"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -I$PKG/csrc $fl -c -o $TMP/${f%.hip}.o $src &
  objs+=($TMP/${f%.hip}.o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT "${objs[@]}"
rm -rf $TMP
echo built $OUT
