#!/usr/bin/env bash
# Config 4 brick marches: XCD-aware brick order (B, the new default) vs plain order (A,
# tools/build/libtvam_base4.so), interleaved timings on a 40-angle shard, then FETCH / TCC counters
# of both.  usage: tools/runs/r05_binxcd.sh OUT
set -o pipefail
o=$1; mkdir -p $o/a $o/b
export TMPDIR=/tmp
for r in 1 2; do
  TVAM_LIB=tools/build/libtvam_base4.so timeout -k 10 200 python3 -u tools/profile_jitter.py 4 400 40 2 >> $o/time_a.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/profile_jitter.py 4 400 40 2 >> $o/time_b.log 2>&1 || exit 1
done
for v in a b; do
  lib=drtvam_amd/libtvam.so; [ $v = a ] && lib=tools/build/libtvam_base4.so
  i=0
  for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    TVAM_LIB=$lib timeout -k 10 -s KILL 240 rocprofv3 --pmc $set -d $o/$v/p$i -o p --output-format csv -- python3 tools/profile_jitter.py 4 400 40 > $o/$v/p$i.log 2>&1 || exit 1
  done
  echo "variant $v" >> $o/summary.txt
  python3 tools/pmc_summary.py $o/$v >> $o/summary.txt
done
