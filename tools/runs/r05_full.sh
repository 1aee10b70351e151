#!/usr/bin/env bash
# the whole -m gpu suite, then the default bench line and its kernel stats. usage: tools/runs/r05_full.sh OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
tools/runs/r05_bench.sh $o/bench || exit 1
exit $rc
