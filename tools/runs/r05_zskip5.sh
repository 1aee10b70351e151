#!/usr/bin/env bash
# Tile adjoint skipping all-zero gradient tiles: config 5 and config 4 bench lines, current vs
# tools/build/libtvam_noskip.so, interleaved.  usage: OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for v in cur noskip; do
  lib=drtvam_amd/libtvam.so; [ $v = noskip ] && lib=tools/build/libtvam_$v.so
  TVAM_LIB=$lib timeout -k 10 300 python bench.py --config 5 --n 800 --steps 3 --warmup 1 --cpu-baseline off > $o/c5_$v.json 2>> $o/err.log || exit 1
  TVAM_LIB=$lib timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --cpu-baseline off > $o/c4_$v.json 2>> $o/err.log || exit 1
  TVAM_LIB=$lib timeout -k 10 200 python bench.py --cpu-baseline off > $o/c2_$v.json 2>> $o/err.log || exit 1
done
