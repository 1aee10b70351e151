#!/usr/bin/env bash
# A/B of env switches on tools/profile_jitter.py runs, then selected tests and benches.
# usage (GPU box): tools/ab_env.sh OUT "ENV=A ENV=B" "PROFILE ARGS|..." "TEST FILES" "BENCH ARGS|..."
set -o pipefail
o=$1; mkdir -p $o
IFS='|' read -ra P <<< "$3"
i=0
for pa in "${P[@]}"; do
  i=$((i+1))
  for ev in $2; do
    env $ev timeout -k 10 200 python tools/profile_jitter.py $pa > $o/p${i}_${ev}.log 2>&1 || exit 1
  done
done
if [ -n "$4" ]; then
  timeout -k 10 900 python -u -m pytest $4 -m gpu -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
fi
IFS='|' read -ra B <<< "$5"
i=0
for b in "${B[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $b --cpu-baseline off > $o/bench$i.json 2> $o/bench$i.err || exit 1
done
