#!/usr/bin/env bash
# Angle-shard readiness of configs 4 and 5: every rank of an 8-rank angle
# shard timed on this one GPU (bench.py --emulate R/8 --shard angle: no collectives; the RCCL
# dose all-reduce enters through the record's cost model), plus config 5 with filter_radon
# (item 8).  usage (GPU box, repo root): tools/emulate_angle8.sh OUT [configs...]
set -euo pipefail
out="$1"; shift; mkdir -p "$out"
cfgs="${*:-4 5}"
for c in $cfgs; do
  n=400; [ "$c" = 5 ] && n=800
  for r in 0 1 2 3 4 5 6 7; do
    cmd="python bench.py --config $c --n $n --emulate $r/8 --shard angle --steps 2 --warmup 1 --prewarm 0"
    timeout -k 10 300 $cmd > "$out/c${c}_r$r.json" 2>> "$out/emulate.err"
    sed "s|^{|{\"cmd\": \"$cmd\", |" "$out/c${c}_r$r.json" >> "$out/emulate_angle8.jsonl"
    echo "config $c rank $r done" >&2
  done
done
