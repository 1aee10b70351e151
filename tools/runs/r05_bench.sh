#!/usr/bin/env bash
# bench line + rocprofv3 kernel stats of the same command. usage: tools/runs/r05_bench.sh OUT [bench args]
set -o pipefail
o=$1; shift; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --cpu-baseline off "$@" > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o k --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline off "$@" > $o/trace_bench.json 2> $o/trace_bench.err || exit 1
