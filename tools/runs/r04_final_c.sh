#!/usr/bin/env bash
# Round-4 record, part C: bench lines of configs 3 / 4 / 5 (+ filter_radon), the 8-rank angle-shard
# emulation of config 4 and the z-slab emulation of config 2.  usage: tools/runs/r04_final_c.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config 3 --cpu-baseline off > "$o/bench_config3.json" 2> "$o/bench_config3.err"
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config4.json" 2> "$o/bench_config4.err"
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config5.json" 2> "$o/bench_config5.err"
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --filter-radon --cpu-baseline off \
  > "$o/bench_config5_filter_radon.json" 2> "$o/bench_config5_filter_radon.err"
tools/emulate_angle8.sh "$o/emulate_c4" 4
tools/scale_emulate.sh "$o/emulate_slab"
