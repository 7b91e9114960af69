#!/bin/bash
# Build libipls_agg.so of git revision REV (default HEAD) into OUT (default
# ipls-java-api_amd/lib/ab/libipls_agg_REV.so), for same-box A/B runs of the
# library (load it with IPLS_AGG_LIB=OUT).  Dev tool, not the product.
set -euo pipefail
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${2:-$R/ipls-java-api_amd/lib/ab/libipls_agg_$(git -C "$R" rev-parse --short "$REV").so}
T=$(mktemp -d)
git -C "$R" archive "$REV" ipls-java-api_amd/csrc include | tar -x -C "$T"
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I"$T/include" \
  -shared -Wl,--version-script="$T/ipls-java-api_amd/csrc/exports.map" -o "$OUT" \
  "$T"/ipls-java-api_amd/csrc/ipls_agg.cpp "$T"/ipls-java-api_amd/csrc/engine.hip \
  "$T"/ipls-java-api_amd/csrc/pubsub_host.cpp "$T"/ipls-java-api_amd/csrc/javaser.cpp
rm -rf "$T"
echo "built $OUT from $REV"
