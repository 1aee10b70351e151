#!/usr/bin/env bash
# Round-5 record, part A: counters of configs 2 and 3 (tools/pmc_bench.sh), the default bench line
# (config 2, with the CPU baseline) and the rocprofv3 kernel stats of the same command.
# usage: tools/runs/r05_final_a.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
tools/pmc_bench.sh "$o/pmc_c2" 2
tools/pmc_bench.sh "$o/pmc_c3" 3
timeout -k 10 300 python bench.py > "$o/bench.json" 2> "$o/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/prof" -o k --output-format csv -- \
  python3 bench.py --cpu-baseline off > "$o/bench_under_rocprof.json" 2> "$o/bench_under_rocprof.err"
