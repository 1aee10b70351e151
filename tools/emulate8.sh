#!/usr/bin/env bash
# Every rank of an 8-rank config-2 run, emulated one shard at a time on this GPU (bench.py --emulate
# R/8: no collectives; the angle split's RCCL dose all-reduces enter through the record's cost
# model).  usage (GPU box, repo root): tools/emulate8.sh OUT [slab|angle ...]
set -euo pipefail
out="$1"; shift; mkdir -p "$out"
for sh in "${@:-slab angle}"; do
  for r in 0 1 2 3 4 5 6 7; do
    cmd="python bench.py --config 2 --emulate $r/8 --shard $sh --steps 20 --warmup 2"
    timeout -k 10 180 $cmd > "$out/${sh}_r$r.json" 2>> "$out/emulate.err"
    sed "s|^{|{\"cmd\": \"$cmd\", |" "$out/${sh}_r$r.json" >> "$out/emulate_${sh}8.jsonl"
    echo "$sh rank $r done" >&2
  done
done
