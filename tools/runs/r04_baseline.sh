#!/usr/bin/env bash
# Round-4 baseline on the GPU box: HEAD's config-2 and config-4 bench lines, and fresh counters
# (tools/pmc_bench.sh) of configs 4 and 5.  usage: tools/runs/r04_baseline.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --cpu-baseline off > "$o/bench_c2.json" 2> "$o/bench_c2.err"
timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --cpu-baseline off > "$o/bench_c4.json" 2> "$o/bench_c4.err"
tools/pmc_bench.sh "$o/pmc_c4" 4
tools/pmc_bench.sh "$o/pmc_c5" 5 800
