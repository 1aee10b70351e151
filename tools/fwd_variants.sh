#!/usr/bin/env bash
# Planar forward / adjoint variants on config 2 (kernel_sweep timings).  usage: OUT "ENV..." ...
set -euo pipefail
out="$1"; shift; mkdir -p "$out"
for v in "$@"; do
  echo "== $v" >> "$out/var.log"
  env $v timeout -k 10 120 python tools/kernel_sweep.py 400 0 >> "$out/var.log" 2>&1
done
