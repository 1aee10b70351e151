#!/usr/bin/env bash
# Jittered / stray-list parity suites, then config 5 and config 4 bench lines (GPU box, repo root)
set -o pipefail
o=gpurun_out/a3; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_square.py tests/test_gpu_baseline_sizes.py tests/test_gpu_edge_cases.py tests/test_gpu_cylindrical.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_config5.json 2> $o/bench_config5.err || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_config4.json 2> $o/bench_config4.err || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof5 -o k --output-format csv -- python3 bench.py --config 5 --n 800 --steps 1 --warmup 0 --cpu-baseline off > $o/c5_rocprof.json 2> $o/c5_rocprof.err
