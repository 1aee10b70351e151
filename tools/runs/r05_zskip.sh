#!/usr/bin/env bash
# List adjoint skipping all-zero gradient tiles (current) vs marching them (tools/build/libtvam_noskip.so):
# config 2 bench lines, interleaved.  usage: OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur noskip; do
    lib=drtvam_amd/libtvam.so; [ $v = noskip ] && lib=tools/build/libtvam_$v.so
    TVAM_LIB=$lib timeout -k 10 200 python bench.py --cpu-baseline off > $o/${v}_$r.json 2>> $o/err.log || exit 1
  done
done
