#!/usr/bin/env bash
# Round 4: bench lines of configs 2 / 4 / 5 with the current defaults, then the whole -m gpu suite.
# usage: tools/runs/r04_ab4.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --cpu-baseline off > "$o/c2.json" 2> "$o/c2.err"
timeout -k 10 200 python bench.py --config 4 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c4.json" 2> "$o/c4.err"
timeout -k 10 200 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c5.json" 2> "$o/c5.err"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$o/tests.log" 2>&1
