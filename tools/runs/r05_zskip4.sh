#!/usr/bin/env bash
# Brick-march adjoint skipping all-zero gradient bricks: config 4 bench lines, current vs
# tools/build/libtvam_binnoskip.so (the tile-adjoint skip in both), then the scattering GPU tests.
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for v in cur binnoskip; do
  lib=drtvam_amd/libtvam.so; [ $v = binnoskip ] && lib=tools/build/libtvam_$v.so
  TVAM_LIB=$lib timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --cpu-baseline off > $o/c4_$v.json 2>> $o/err.log || exit 1
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scattering.py tests/test_gpu_bin_chunks.py -k "not config5" > $o/tests.log 2>&1 || exit 1
