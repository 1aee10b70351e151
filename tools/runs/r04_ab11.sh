#!/usr/bin/env bash
# Round 4: configs 5 and 4 (sample-fastest adjoint groups) and config 2 (pipelined L-BFGS direction) against HEAD.
# usage: tools/runs/r04_ab11.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
c4="--config 4 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off"
c5="--config 5 --n 800 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off"
(cd _variants/head && timeout -k 10 240 python bench.py $c5) > "$o/c5_head.json" 2> "$o/c5_head.err"
timeout -k 10 240 python bench.py $c5 > "$o/c5_new.json" 2> "$o/c5_new.err"
(cd _variants/head && timeout -k 10 240 python bench.py $c5) > "$o/c5_head2.json" 2> "$o/c5_head2.err"
timeout -k 10 240 python bench.py $c5 > "$o/c5_new2.json" 2> "$o/c5_new2.err"
(cd _variants/head && timeout -k 10 240 python bench.py $c4) > "$o/c4_head.json" 2> "$o/c4_head.err"
timeout -k 10 240 python bench.py $c4 > "$o/c4_new.json" 2> "$o/c4_new.err"
TVAM_BIN_CBITS=2 timeout -k 10 240 python bench.py $c4 > "$o/c4_new_cbits2.json" 2> "$o/c4_new_cbits2.err"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_pipeline.py tests/test_gpu_lbfgs.py > "$o/tests_pipeline.log" 2>&1
c2="--steps 20 --warmup 2 --cpu-baseline off"
timeout -k 10 150 python bench.py $c2 > "$o/c2_new.json" 2> "$o/c2_new.err"
(cd _variants/head && timeout -k 10 150 python bench.py $c2) > "$o/c2_head.json" 2> "$o/c2_head.err"
timeout -k 10 150 python bench.py $c2 > "$o/c2_new2.json" 2> "$o/c2_new2.err"
(cd _variants/head && timeout -k 10 150 python bench.py $c2) > "$o/c2_head2.json" 2> "$o/c2_head2.err"
