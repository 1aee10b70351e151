#!/usr/bin/env bash
# Thin-slab list adjoint: 16- vs 8-slice chunks on the 8-rank (50-slice) and 4-rank (100-slice) slabs.
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for rw in 3/8 0/4; do
    for z in 16 8; do
      TVAM_EXPERIMENTAL=1 TVAM_ADJL_Z=$z timeout -k 10 120 python bench.py --emulate $rw --shard slab --steps 10 --warmup 2 --cpu-baseline off | sed "s/^{/{\"adjl_z\": $z, /" >> $o/emu.jsonl 2>> $o/err.log || exit 1
    done
  done
done
