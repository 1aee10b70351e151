#!/usr/bin/env bash
# Round record on the GPU box: the whole -m gpu suite, smoke(), the default bench line (config 2)
# and the rocprofv3 kernel stats of the same bench command.  usage: tools/round_final.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > "$o/gpu_tests.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$o/smoke.log" 2>&1
timeout -k 10 300 python bench.py > "$o/bench.json" 2> "$o/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/prof" -o k --output-format csv -- \
  python3 bench.py --cpu-baseline off > "$o/bench_under_rocprof.json" 2> "$o/bench_under_rocprof.err"
