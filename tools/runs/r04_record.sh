#!/usr/bin/env bash
# Round-4 record on the final build, one part per GPU call:
#   a: counters of configs 2 and 3 (tools/pmc_bench.sh), the default bench line (config 2, with the
#      CPU baseline) and the rocprofv3 kernel stats of the same command;
#   b: counters of configs 4 and 5;
#   c: bench lines of configs 3 / 4 / 5 (+ filter_radon), the 8-rank angle-shard emulation of
#      config 4 and the z-slab emulation of config 2;
#   d: the whole -m gpu suite, smoke() and the default bench line again (with every summary current);
#   f: bench lines of configs 3 / 4 / 5 (+ filter_radon) and the z-slab emulation of config 2
#      (run after the summaries of a and b are committed, so the lines carry live rooflines).
# usage: tools/runs/r04_record.sh PART OUT
set -euo pipefail
part="$1"; o="$(realpath -m "$2")"; mkdir -p "$o"
export TMPDIR=/tmp
case "$part" in
  a)
    tools/pmc_bench.sh "$o/pmc_c2" 2
    tools/pmc_bench.sh "$o/pmc_c3" 3
    timeout -k 10 300 python bench.py > "$o/bench.json" 2> "$o/bench.err"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$o/prof" -o k --output-format csv -- \
      python3 bench.py --cpu-baseline off > "$o/bench_under_rocprof.json" 2> "$o/bench_under_rocprof.err"
    ;;
  b)
    tools/pmc_bench.sh "$o/pmc_c4" 4
    tools/pmc_bench.sh "$o/pmc_c5" 5 800
    ;;
  c)
    timeout -k 10 300 python bench.py --config 3 --cpu-baseline off > "$o/bench_config3.json" 2> "$o/bench_config3.err"
    timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config4.json" \
      2> "$o/bench_config4.err"
    timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --cpu-baseline off \
      > "$o/bench_config5.json" 2> "$o/bench_config5.err"
    timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --filter-radon --cpu-baseline off \
      > "$o/bench_config5_filter_radon.json" 2> "$o/bench_config5_filter_radon.err"
    tools/emulate_angle8.sh "$o/emulate_c4" 4
    tools/scale_emulate.sh "$o/emulate_slab"
    ;;
  f)
    timeout -k 10 300 python bench.py --config 3 --cpu-baseline off > "$o/bench_config3.json" 2> "$o/bench_config3.err"
    timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 1 --cpu-baseline off > "$o/bench_config4.json" \
      2> "$o/bench_config4.err"
    timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --cpu-baseline off \
      > "$o/bench_config5.json" 2> "$o/bench_config5.err"
    timeout -k 10 300 python bench.py --config 5 --n 800 --steps 5 --warmup 1 --filter-radon --cpu-baseline off \
      > "$o/bench_config5_filter_radon.json" 2> "$o/bench_config5_filter_radon.err"
    tools/scale_emulate.sh "$o/emulate_slab"
    ;;
  d)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
      > "$o/gpu_tests.log" 2>&1
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$o/smoke.log" 2>&1
    timeout -k 10 300 python bench.py > "$o/bench.json" 2> "$o/bench.err"
    for b in 2 3 4; do  # the opt-in banded iteration at 2 / 3 / 4 slab bands, same box
      timeout -k 10 150 python bench.py --slab-bands $b --cpu-baseline off > "$o/bench_bands$b.json" 2> "$o/bench_bands$b.err"
    done
    ;;
esac
