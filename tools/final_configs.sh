#!/usr/bin/env bash
# Bench lines of configs 3-5 on the final build, each with the rocprofv3 kernel stats of the same
# command (raw traces deleted).  usage (GPU box, repo root): tools/final_configs.sh OUT
set -euo pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $o/bench_$name.json 2> $o/bench_$name.err
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/prof_$name -o k --output-format csv -- \
    python3 bench.py "$@" > $o/bench_${name}_under_rocprof.json 2> $o/bench_${name}_under_rocprof.err
  cp $o/prof_$name/k_kernel_stats.csv $o/bench_${name}_kernel_stats.csv
  rm -rf $o/prof_$name
  echo "$name done" >&2
}
run config3 --config 3 --cpu-baseline off
run config4 --config 4 --steps 2 --warmup 1 --cpu-baseline off
run config5 --config 5 --n 800 --steps 2 --warmup 1 --cpu-baseline off
timeout -k 10 400 python3 bench.py --config 5 --n 800 --steps 2 --warmup 1 --cpu-baseline off --filter-radon > $o/bench_config5_filter_radon.json 2> $o/bench_config5_filter_radon.err
