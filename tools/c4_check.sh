#!/usr/bin/env bash
# Config-4 change check (GPU box): scattering / bin-chunk parity tests, the config-4 bench line and
# a rocprofv3 kernel-stats pass of a short bench run.  usage: tools/c4_check.sh OUT [pytest files]
set -euo pipefail
o="$1"; shift; mkdir -p "$o"
export TMPDIR=/tmp
files="${*:-tests/test_gpu_scattering.py tests/test_gpu_bin_chunks.py}"
timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 600 --timeout-method thread > "$o/tests.log" 2>&1
timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --cpu-baseline off > "$o/bench4.json" 2> "$o/bench4.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$o/prof" -o k --output-format csv -- \
  python3 bench.py --config 4 --steps 2 --warmup 0 --prewarm 0 --cpu-baseline off > "$o/prof.log" 2>&1
