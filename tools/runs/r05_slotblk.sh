#!/usr/bin/env bash
# Config 5 slot orders (200-angle shard): length classes over all angles (TVAM_SLOT_SORT=2, the
# default) vs classes within blocks of B angles (TVAM_SLOT_SORT=3), interleaved.  usage: OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp TVAM_EXPERIMENTAL=1
for r in 1 2; do
  for v in "2 0" "3 4" "3 16" "3 64"; do
    set -- $v
    echo "sort $1 block $2" >> $o/time.log
    TVAM_SLOT_SORT=$1 TVAM_SLOT_BLOCK=$2 timeout -k 10 200 python3 -u tools/profile_jitter.py 5 800 200 2 >> $o/time.log 2>&1 || exit 1
  done
done
