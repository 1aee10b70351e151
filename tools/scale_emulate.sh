#!/usr/bin/env bash
# Per-rank compute time of W-rank runs, emulated one shard at a time on one GPU
# (bench.py --emulate R/W: no collectives).  usage: tools/scale_emulate.sh OUT [Z...]
set -euo pipefail
out="$1"; shift; mkdir -p "$out"
for rw in 0/1 0/2 0/4 0/8 3/8; do
  timeout -k 10 120 python bench.py --emulate $rw --steps 10 --warmup 2 >> "$out/emulate.jsonl" 2>> "$out/emulate.err"
done
for z in "$@"; do
  for rw in 0/4 0/8; do
    TVAM_PLANAR_FWD_Z=$z timeout -k 10 120 python bench.py --emulate $rw --steps 10 --warmup 2 | sed "s/^{/{\"fwd_z\": $z, /" >> "$out/emulate.jsonl" 2>> "$out/emulate.err"
  done
done
