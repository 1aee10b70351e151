#!/usr/bin/env bash
# Round 4: the 16-byte pattern binning (tvam_slice_bin4_kernel) against the one-float kernel
# (TVAM_SLICE_BIN1=1) on one box: its tests, then configs 2 and 3.  usage: tools/runs/r04_ab13.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_slice_bin.py tests/test_gpu_parity.py tests/test_gpu_fwd_pairs.py tests/test_gpu_pipeline.py \
  > "$o/tests.log" 2>&1
c2="--steps 20 --warmup 2 --cpu-baseline off"
for r in 1 2; do
  timeout -k 10 150 python bench.py $c2 > "$o/c2_new_$r.json" 2> "$o/c2_new_$r.err"
  TVAM_SLICE_BIN1=1 timeout -k 10 150 python bench.py $c2 > "$o/c2_old_$r.json" 2> "$o/c2_old_$r.err"
done
timeout -k 10 150 python bench.py --config 3 --cpu-baseline off > "$o/c3_new.json" 2> "$o/c3_new.err"
TVAM_SLICE_BIN1=1 timeout -k 10 150 python bench.py --config 3 --cpu-baseline off > "$o/c3_old.json" 2> "$o/c3_old.err"
