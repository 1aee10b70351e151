#!/usr/bin/env bash
# Round 4: the adjoint tile kernel with sample-fastest groups (one global atomic per pixel and tile)
# against HEAD (_variants/head): jittered-adjoint parity tests, then configs 4 and 5.
# usage: tools/runs/r04_ab10.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_square.py tests/test_gpu_active_set.py tests/test_gpu_cylindrical.py \
  tests/test_gpu_estimators.py tests/test_gpu_scattering.py tests/test_gpu_distributed.py > "$o/tests.log" 2>&1
c4="--config 4 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off"
c5="--config 5 --n 800 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off"
timeout -k 10 240 python bench.py $c4 > "$o/c4_new.json" 2> "$o/c4_new.err"
(cd _variants/head && timeout -k 10 240 python bench.py $c4) > "$o/c4_head.json" 2> "$o/c4_head.err"
timeout -k 10 240 python bench.py $c5 > "$o/c5_new.json" 2> "$o/c5_new.err"
(cd _variants/head && timeout -k 10 240 python bench.py $c5) > "$o/c5_head.json" 2> "$o/c5_head.err"
TVAM_BIN_CBITS=2 timeout -k 10 240 python bench.py $c4 > "$o/c4_new_cbits2.json" 2> "$o/c4_new_cbits2.err"
