#!/usr/bin/env bash
# Config 5 tile edge after the XCD-local slice order: 73 (default) vs 62 / 80 / 89 on 200 angles.
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for t in 0 80 89 62; do
    echo "tile $t" >> $o/time.log
    PJ_TILE=$t timeout -k 10 200 python3 -u tools/profile_jitter.py 5 800 200 2 >> $o/time.log 2>&1 || exit 1
  done
done
