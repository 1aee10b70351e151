#!/usr/bin/env bash
# Round-5 record, part C: the default bench line (config 2, CPU baseline) and the rocprofv3 kernel
# stats of the same command, bench lines of configs 3 / 4 / 5 (+ filter_radon) and the z-slab emulation of config 2.
# usage: tools/runs/r05_final_c.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > "$o/bench.json" 2> "$o/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/prof" -o k --output-format csv -- \
  python3 bench.py > "$o/bench_under_rocprof.json" 2> "$o/bench_under_rocprof.err"
timeout -k 10 300 python bench.py --config 3 --cpu-baseline off > "$o/bench_config3.json" 2> "$o/bench_config3.err"
timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config4.json" 2> "$o/bench_config4.err"
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config5.json" 2> "$o/bench_config5.err"
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --filter-radon --cpu-baseline off \
  > "$o/bench_config5_filter_radon.json" 2> "$o/bench_config5_filter_radon.err"
tools/scale_emulate.sh "$o/emulate_slab"
