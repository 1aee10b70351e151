#!/usr/bin/env bash
# Round 4: the parity tests of the kernels changed this round.  usage: tools/runs/r04_tests1.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scattering.py \
  tests/test_gpu_bin_chunks.py tests/test_gpu_parity.py tests/test_gpu_square.py tests/test_gpu_active_set.py \
  tests/test_gpu_distributed.py tests/test_gpu_bench.py tests/test_gpu_baseline_sizes.py > "$o/tests.log" 2>&1
