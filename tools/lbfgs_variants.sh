#!/usr/bin/env bash
# tools/lbfgs_sweep.py under env variants.  usage: OUT "ENV..." ...
set -euo pipefail
out="$1"; shift; mkdir -p "$out"
for v in "$@"; do
  env $v timeout -k 10 120 python tools/lbfgs_sweep.py >> "$out/lbfgs.log"
done
