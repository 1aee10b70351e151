#!/usr/bin/env bash
# Refracted forward with 24-byte column records: cylindrical / baseline-size / parity suites, config 3 bench + stats
set -o pipefail
o=gpurun_out/a13; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cylindrical.py tests/test_gpu_baseline_sizes.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 3 --cpu-baseline off > $o/bench_config3.json 2> $o/bench_config3.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof3 -o k --output-format csv -- python3 bench.py --config 3 --steps 5 --cpu-baseline off > $o/c3_rocprof.json 2> $o/c3_rocprof.err
