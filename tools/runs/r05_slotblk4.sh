#!/usr/bin/env bash
# Config 4 (40-angle shard) slot orders: TVAM_SLOT_SORT=2 vs 3 (classes within blocks of 16 angles), interleaved.
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp TVAM_EXPERIMENTAL=1
for r in 1 2; do
  for v in 2 3; do
    echo "sort $v" >> $o/time4.log
    TVAM_SLOT_SORT=$v TVAM_SLOT_BLOCK=16 timeout -k 10 200 python3 -u tools/profile_jitter.py 4 400 40 2 >> $o/time4.log 2>&1 || exit 1
  done
done
