#!/usr/bin/env bash
# A/B of the per-ray tile kernels' slot order (TVAM_SLOT_SORT 1: within angle, 2: length classes)
# on config 5 / 4a angle shards, then the config-5 bench.  usage (GPU box): tools/ab_slot_sort.sh OUT
set -o pipefail
o=$1; mkdir -p $o
for c in 1 2; do
  TVAM_SLOT_SORT=$c timeout -k 10 150 python tools/profile_jitter.py 5 800 80 3 > $o/c5_sort$c.log 2>&1 || exit 1
  TVAM_SLOT_SORT=$c timeout -k 10 120 python tools/profile_jitter.py 4a 400 40 3 > $o/c4a_sort$c.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_c5.json 2> $o/bench_c5.err || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_square.py tests/test_gpu_baseline_sizes.py -m gpu -x -v --timeout 200 --timeout-method thread > $o/tests.log 2>&1
