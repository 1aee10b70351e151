#!/usr/bin/env bash
# Build a variant libtvam.so into _variants/: tvam_planar.hip (or $SRC) compiled with extra flags,
# the other translation units from a cached default build.
# usage: tools/build_variant.sh NAME "-DFLAG=V ..." [src]
set -euo pipefail
here="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; vflags="$2"; vsrc="${3:-tvam_planar}"
cs="$here/drtvam_amd/csrc"
cache="$here/_variants/obj"
mkdir -p "$cache" "$here/_variants"
flags=(--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt
       -munsafe-fp-atomics -Wall -Wno-unused-function -I"$here/include")
objs=()
for src in tvam_plan tvam_kernels tvam_planar tvam_adjlist tvam_vec tvam_scatter tvam_radon; do
  if [ "$src" = "$vsrc" ]; then
    o="$cache/${src}_$name.o"
    /opt/rocm/bin/hipcc "${flags[@]}" $vflags -c "$cs/$src.hip" -o "$o"
  else
    o="$cache/$src.o"
    if [ ! -f "$o" ] || [ "$cs/$src.hip" -nt "$o" ] || [ "$cs/tvam_internal.h" -nt "$o" ]; then
      /opt/rocm/bin/hipcc "${flags[@]}" -c "$cs/$src.hip" -o "$o"
    fi
  fi
  objs+=("$o")
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$here/_variants/libtvam_$name.so"
echo "built _variants/libtvam_$name.so"
