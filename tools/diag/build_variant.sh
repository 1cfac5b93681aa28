#!/bin/bash
# Build a diagnostic copy of the codec library: tools/diag/variants/lib_<name>.so from the
# working tree (or from git ref <ref>) with extra compiler flags.  Timing A/B only; never shipped.
#   tools/diag/build_variant.sh <name> "<flags>" [<git ref>]
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
name=$1; flags=$2; ref=$3
out=$ROOT/tools/diag/variants
mkdir -p "$out"
src=$ROOT
if [ -n "$ref" ]; then
  src=$(mktemp -d)
  (cd "$ROOT" && git archive "$ref" decentralizepy_amd/csrc include) | tar -x -C "$src"
fi
cd "$src/decentralizepy_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off $flags -shared \
  -o "$out/lib_$name.so" dpz_*.hip dpz_batch.cpp -lhipfft
echo "built $out/lib_$name.so"
