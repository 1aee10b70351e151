#!/usr/bin/env bash
# Sparse-set ray-record reuse: active-set / distributed / radon / occlusion suites, config 5 filter_radon bench
set -o pipefail
o=gpurun_out/a12; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_active_set.py tests/test_gpu_distributed.py tests/test_gpu_radon.py "tests/test_gpu_optimization.py::test_box_hole_occlusion_optimization" -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --filter-radon --cpu-baseline off > $o/bench_config5_filter_radon.json 2> $o/bench_config5_filter_radon.err
