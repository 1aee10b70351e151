#!/usr/bin/env bash
# Planar adjoint variants on config 2 (kernel_sweep over tile sizes) under env
# variants.  usage: OUT "TILES" "ENV..." ...
set -euo pipefail
out="$1"; tiles="$2"; shift 2; mkdir -p "$out"
for v in "$@"; do
  echo "== $v" >> "$out/var.log"
  env $v timeout -k 10 200 python tools/kernel_sweep.py 400 $tiles >> "$out/var.log" 2>&1
done
