#!/usr/bin/env bash
# Host build + run of tools/brick_count_check.hip (no GPU needed).  usage: tools/brick_count_check.sh [N]
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
out="${TMPDIR:-/tmp}/brick_count_check"
/opt/rocm/bin/hipcc -O2 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I"$here/../include" \
  "$here/brick_count_check.hip" -o "$out"
"$out" "${1:-2000000}"
