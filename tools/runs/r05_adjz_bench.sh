#!/usr/bin/env bash
# Config 2 bench with the list adjoint at 16 (default) vs 8 slices per workgroup, interleaved.
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for z in 16 8; do
    TVAM_EXPERIMENTAL=1 TVAM_ADJL_Z=$z timeout -k 10 200 python bench.py --cpu-baseline off > $o/z${z}_$r.json 2>> $o/err.log || exit 1
  done
done
