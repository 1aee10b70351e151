#!/usr/bin/env bash
# Round 4: the optimiser iteration in slab bands (pipelined projections / vector passes): its GPU
# tests, then config 2 against HEAD (_variants/head), twice.  usage: tools/runs/r04_ab12.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_pipeline.py tests/test_gpu_lbfgs.py tests/test_gpu_distributed.py tests/test_gpu_optimization.py \
  > "$o/tests.log" 2>&1
c2="--steps 20 --warmup 2 --cpu-baseline off"
timeout -k 10 150 python bench.py $c2 > "$o/c2_new.json" 2> "$o/c2_new.err"
(cd _variants/head && timeout -k 10 150 python bench.py $c2) > "$o/c2_head.json" 2> "$o/c2_head.err"
timeout -k 10 150 python bench.py $c2 > "$o/c2_new2.json" 2> "$o/c2_new2.err"
(cd _variants/head && timeout -k 10 150 python bench.py $c2) > "$o/c2_head2.json" 2> "$o/c2_head2.err"
