#!/bin/bash
# Build tools/ab_sweep.hip against the kernels of git revision REV (default
# HEAD) renamed into namespace ipls_old.  Output: ipls-java-api_amd/lib/ab_sweep
set -euo pipefail
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" show "$REV:ipls-java-api_amd/csrc/ipls_kernels.hpp" |
  sed 's/^namespace ipls {/namespace ipls_old {/; s|^}  // namespace ipls$|}  // namespace ipls_old|' > "$T/ipls_kernels_old.hpp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math ${AB_FLAGS:-} \
  -DAB_OLD_HEADER="\"$T/ipls_kernels_old.hpp\"" -o "$R/ipls-java-api_amd/lib/ab_sweep" "$R/tools/ab_sweep.hip"
rm -rf "$T"
echo "built ab_sweep: new = working tree, old = $REV"
