#!/usr/bin/env bash
# Counter passes (tools/pmc_bench.sh) of the BASELINE configs' bench iterations, one after the other.
# usage (GPU box, repo root): tools/pmc_configs.sh OUT CONFIG...
set -euo pipefail
out="$1"; shift
for c in "$@"; do
  n=400; [ "$c" = 5 ] && n=800
  bash tools/pmc_bench.sh "$out/c$c" "$c" "$n"
  echo "config $c counters done" >&2
done
