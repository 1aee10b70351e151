#!/usr/bin/env bash
# Round-4 record, part E: bench lines of configs 4 and 5 with their current counter summaries,
# and config 2 at 1 / 2 / 3 / 4 slab bands (the opt-in banded iteration), same box.
# usage: tools/runs/r04_final_e.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config4.json" \
  2> "$o/bench_config4.err"
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --cpu-baseline off \
  > "$o/bench_config5.json" 2> "$o/bench_config5.err"
for b in 1 2 3 4; do
  timeout -k 10 150 python bench.py --slab-bands $b --cpu-baseline off > "$o/bench_bands$b.json" 2> "$o/bench_bands$b.err"
done
