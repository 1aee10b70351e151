#!/usr/bin/env bash
# Adjoint partials sorted by pixel: scattering parity suites, config-4 shard kernel stats, config 4 bench
set -o pipefail
o=gpurun_out/a14; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scattering.py tests/test_gpu_bin_chunks.py tests/test_gpu_surface.py -x -v -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/shard -o k --output-format csv -- python3 tools/profile_jitter.py 4 400 40 2 > $o/shard.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_config4.json 2> $o/bench_config4.err
