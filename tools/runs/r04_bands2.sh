#!/usr/bin/env bash
# Round 4: the banded iteration with the gradient zeroed once (Python only), config 2 at 1 / 2 / 3
# slab bands twice each on one box, and the banded-iteration GPU tests.  usage: tools/runs/r04_bands2.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_pipeline.py > "$o/tests.log" 2>&1
for r in 1 2; do
  for b in 1 2 3; do
    timeout -k 10 150 python bench.py --slab-bands $b --cpu-baseline off > "$o/bands${b}_$r.json" 2> "$o/bands${b}_$r.err"
  done
done
