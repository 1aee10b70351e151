#!/usr/bin/env bash
# bench.py lines (no CPU baseline) under env variants.  usage: OUT CONFIG "ENV..." ...
set -euo pipefail
out="$1"; cfg="$2"; shift 2; mkdir -p "$out"
for v in "$@"; do
  echo "== $v" >> "$out/bench.log"
  env $v timeout -k 10 300 python bench.py --config "$cfg" --steps 5 --warmup 2 --cpu-baseline off 2>/dev/null \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['fwd_ms'], d['config']['adj_ms'])" >> "$out/bench.log"
done
