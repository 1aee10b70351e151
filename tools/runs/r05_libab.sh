#!/usr/bin/env bash
# A/B of two library builds on config 2 (tools/proj_ab.py), interleaved: usage tools/runs/r05_libab.sh OUT LIB_A LIB_B [variant]
set -o pipefail
o=$1; a=$2; b=$3; v=${4:-}
mkdir -p $o
for r in 1 2; do
  TVAM_LIB=$a timeout -k 10 200 python -u tools/proj_ab.py 400 "$v" >> $o/a.jsonl 2>>$o/err.log || exit 1
  TVAM_LIB=$b timeout -k 10 200 python -u tools/proj_ab.py 400 "$v" >> $o/b.jsonl 2>>$o/err.log || exit 1
done
