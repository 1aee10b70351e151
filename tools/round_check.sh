#!/usr/bin/env bash
# GPU check of a change set: selected -m gpu test files, then benches.
# usage (GPU box, repo root): tools/round_check.sh OUT "TEST FILES" "BENCH ARGS|BENCH ARGS|..."
set -o pipefail
o=$1; mkdir -p $o
timeout -k 10 900 python -u -m pytest $2 -m gpu -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
i=0
IFS='|' read -ra B <<< "$3"
for b in "${B[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $b --cpu-baseline off > $o/bench$i.json 2> $o/bench$i.err || exit 1
done
