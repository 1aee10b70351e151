#!/usr/bin/env bash
# Config-4 kernel A/B (GPU box): kernel stats of tools/profile_jitter.py on a 40-angle shard for the
# default library and each variant library given (TVAM_LIB), plus their config-4 bench lines.
# usage: tools/c4_ab.sh OUT [variant.so ...]
set -euo pipefail
o="$1"; shift; mkdir -p "$o"
export TMPDIR=/tmp
i=0
for lib in "" "$@"; do
  i=$((i+1))
  echo "${lib:-default}" > "$o/lib$i.txt"
  TVAM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/t$i" -o k --output-format csv -- \
    python3 tools/profile_jitter.py 4 400 40 2 > "$o/t$i.log" 2>&1
  TVAM_LIB=$lib timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --cpu-baseline off > "$o/bench$i.json" 2> "$o/bench$i.err"
done
