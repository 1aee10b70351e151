#!/usr/bin/env bash
# Build libtvam.so (gfx950) in-tree.  -ffp-contract=off keeps the fp32 ray
# geometry identical to the reference op order (FMAs are written explicitly);
# -munsafe-fp-atomics lowers float atomicAdd to native global/LDS add.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
out="${1:-$here/../libtvam.so}"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
"$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
  -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics \
  -Wall -Wno-unused-function \
  -I"$here/../../include" ${TVAM_CXXFLAGS:-} \
  "$here/tvam_plan.hip" "$here/tvam_kernels.hip" "$here/tvam_planar.hip" "$here/tvam_vec.hip" "$here/tvam_scatter.hip" "$here/tvam_radon.hip" \
  -o "$out"
