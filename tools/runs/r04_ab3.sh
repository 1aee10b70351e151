#!/usr/bin/env bash
# Round 4: kernel stats of config 4 with the counting-sort bins and with the radix-sort path,
# then the whole -m gpu suite.  usage: tools/runs/r04_ab3.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/c4_csort" -o k --output-format csv -- \
  python3 bench.py --config 4 --steps 1 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c4_csort.json" 2> "$o/c4_csort.err"
TVAM_BIN_SORT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/c4_radix" -o k --output-format csv -- \
  python3 bench.py --config 4 --steps 1 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c4_radix.json" 2> "$o/c4_radix.err"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$o/tests.log" 2>&1
