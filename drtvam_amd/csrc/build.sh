#!/usr/bin/env bash
# Build libtvam.so (gfx950) in-tree.  -ffp-contract=off keeps the fp32 ray
# geometry identical to the reference op order (FMAs are written explicitly);
# -munsafe-fp-atomics lowers float atomicAdd to native global/LDS add.
# Each translation unit compiles in parallel (no cross-TU device calls), then one link.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
out="${1:-$here/../libtvam.so}"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
objdir="$(mktemp -d "${TMPDIR:-/tmp}/tvam_build.XXXXXX")"
trap 'rm -rf "$objdir"' EXIT
flags=(--offload-arch=gfx950 -O3 -std=c++17 -fPIC
       -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics
       -Wall -Wno-unused-function -I"$here/../../include")
pids=()
objs=()
for src in tvam_plan tvam_kernels tvam_planar tvam_adjlist tvam_vec tvam_scatter tvam_radon; do
  "$HIPCC" "${flags[@]}" ${TVAM_CXXFLAGS:-} -c "$here/$src.hip" -o "$objdir/$src.o" &
  pids+=($!)
  objs+=("$objdir/$src.o")
done
fail=0
for pid in "${pids[@]}"; do wait "$pid" || fail=1; done
[ "$fail" = 0 ] || { echo "build.sh: compilation failed" >&2; exit 1; }
"$HIPCC" --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$out"
