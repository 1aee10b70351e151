#!/usr/bin/env bash
# Round 4: config 4 with smaller brick-bin chunks (TVAM_BIN_CHUNK_SLOTS): a chunk's records
# (48 B per slot) within the 256 MB Infinity Cache at 4 M slots.  usage: tools/runs/r04_ab7.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
for s in 4194304 16777216 134217728 8388608 33554432; do
  TVAM_BIN_CHUNK_SLOTS=$s timeout -k 10 240 python bench.py --config 4 --steps 2 --warmup 1 --prewarm 0 \
    --cpu-baseline off > "$o/c4_$s.json" 2> "$o/c4_$s.err"
  echo "slots $s done"
done
