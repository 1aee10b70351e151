#!/usr/bin/env bash
# Round 4: kernel trace of the config-2 bench (which small copies run per iteration) and smoke().
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$o/trace" -o k --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --prewarm 0.2 --cpu-baseline off > "$o/bench.json" 2> "$o/bench.err"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$o/smoke.log" 2>&1
