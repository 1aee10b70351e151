#!/usr/bin/env bash
# Tile kernels, slices interleaved over the XCDs (current) vs plain order (TVAM_TILE_XCD=0 build):
# config 5 on 200 angles (tools/profile_jitter.py) and config 5 with filter_radon (bench.py).
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur noxcd; do
    lib=drtvam_amd/libtvam.so; [ $v = noxcd ] && lib=tools/build/libtvam_noxcd.so
    echo "variant $v" >> $o/time.log
    TVAM_LIB=$lib timeout -k 10 200 python3 -u tools/profile_jitter.py 5 800 200 2 >> $o/time.log 2>&1 || exit 1
    TVAM_LIB=$lib timeout -k 10 300 python3 bench.py --config 5 --n 800 --steps 3 --warmup 1 --filter-radon --cpu-baseline off > $o/radon_$v$r.json 2>> $o/err.log || exit 1
  done
done
