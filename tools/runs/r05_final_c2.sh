#!/usr/bin/env bash
# Round-5 record, part C2: rocprofv3 kernel stats of the config 3 / 4 / 5 bench commands of part C
# (the live roofline's launch times against the trace's).  usage: tools/runs/r05_final_c2.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/prof3" -o k --output-format csv -- \
  python3 bench.py --config 3 --cpu-baseline off > "$o/bench_config3.json" 2> "$o/bench_config3.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$o/prof4" -o k --output-format csv -- \
  python3 bench.py --config 4 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config4.json" 2> "$o/bench_config4.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$o/prof5" -o k --output-format csv -- \
  python3 bench.py --config 5 --n 800 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config5.json" 2> "$o/bench_config5.err"
