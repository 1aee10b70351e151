#!/usr/bin/env bash
# Round record on the GPU box: full -m gpu suite, the default bench line (with CPU baseline), and the
# rocprofv3 kernel stats of a bench run.  usage: tools/final_round.sh OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/trace -o bench --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > $o/trace_bench.json 2> $o/trace_bench.err
