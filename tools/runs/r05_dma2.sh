#!/usr/bin/env bash
# Forward LDS-DMA variants on config 2: per-angle table chunk 128 (default) vs 56, and 7 waves per SIMD.
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur ach56 wpe7; do
    lib=tools/build/libtvam_$v.so; [ $v = cur ] && lib=drtvam_amd/libtvam.so
    echo "{\"lib\": \"$v\"}" >> $o/ab.jsonl
    TVAM_LIB=$lib timeout -k 10 200 python -u tools/proj_ab.py 400 >> $o/ab.jsonl 2>>$o/err.log || exit 1
  done
done
