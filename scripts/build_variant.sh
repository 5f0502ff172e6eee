#!/bin/bash
# Build a variant of libvbhem_estep.so for same-box A/B runs (scripts/ab_lib.sh):
#   scripts/build_variant.sh OUT.so [-DFLAG ...] [REPLACEMENT.hip ...]
# Every csrc/*.hip is compiled, except that a REPLACEMENT.hip of the same file name
# takes the place of the tree's source; -D flags go to every compile.
set -e
OUT=$1; shift
PKG=clustering-hidden-markov-models-with-variational-bayesian-hierarchical-em_amd
FLAGS=(); REPL=()
for a in "$@"; do case $a in -D*) FLAGS+=("$a");; *) REPL+=("$(realpath $a)");; esac; done
TMP=$(mktemp -d); objs=()
for src in $PKG/csrc/*.hip; do
  f=$(basename $src); use=$src
  for r in "${REPL[@]}"; do [ "$(basename $r)" = "$f" ] && use=$r; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -I$PKG/csrc "${FLAGS[@]}" -c -o $TMP/${f%.hip}.o $use &
  objs+=($TMP/${f%.hip}.o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT "${objs[@]}"
rm -rf $TMP
echo built $OUT
