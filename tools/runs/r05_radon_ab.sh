#!/usr/bin/env bash
# Config 5 with filter_radon: current build vs the slot classes over all angles (TVAM_SLOT_SORT=2)
# vs plain tile order (TVAM_TILE_XCD=0 build), interleaved.  usage: tools/runs/r05_radon_ab.sh OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in cur sort2 noxcd; do
    lib=drtvam_amd/libtvam.so; env=""
    [ $v = noxcd ] && lib=tools/build/libtvam_noxcd.so
    [ $v = sort2 ] && env="TVAM_EXPERIMENTAL=1 TVAM_SLOT_SORT=2"
    echo "variant $v" >> $o/log.txt
    env TVAM_LIB=$lib $env timeout -k 10 300 python3 bench.py --config 5 --n 800 --steps 3 --warmup 1 --filter-radon --cpu-baseline off > $o/$v$r.json 2>> $o/err.log || exit 1
  done
done
