#!/usr/bin/env bash
# Bench lines of configs 3-5 on the current build (GPU box, repo root): tools/configs_bench.sh OUT
set -o pipefail
o=$1; mkdir -p $o
timeout -k 10 300 python bench.py --config 3 --cpu-baseline off > $o/bench_config3.json 2> $o/bench_config3.err || exit 1
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_config4.json 2> $o/bench_config4.err || exit 1
timeout -k 10 300 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --cpu-baseline off > $o/bench_config5.json 2> $o/bench_config5.err
