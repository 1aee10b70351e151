#!/usr/bin/env bash
# Round 4: kernel trace of config 2's banded iteration (3 slab bands) to see how the two streams
# overlap.  usage: tools/runs/r04_trace_bands.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$o/b3" -o k --output-format csv -- \
  python3 bench.py --slab-bands 3 --steps 4 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/b3.json" 2> "$o/b3.err"
