set -o pipefail
o=gpurun_out/a2; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scattering.py tests/test_gpu_bin_chunks.py -x -v -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_config4.json 2> $o/bench_config4.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof4 -o k --output-format csv -- python3 bench.py --config 4 --steps 1 --warmup 1 --cpu-baseline off > $o/c4_rocprof.json 2> $o/c4_rocprof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof5 -o k --output-format csv -- python3 bench.py --config 5 --n 800 --steps 1 --warmup 1 --cpu-baseline off > $o/c5_rocprof.json 2> $o/c5_rocprof.err
