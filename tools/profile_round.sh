#!/usr/bin/env bash
# Round profile: bench (with CPU baseline), rocprofv3 kernel stats of the bench,
# and HBM traffic counters (separate --pmc passes) of the tile kernels.
# usage (GPU box, repo root): tools/profile_round.sh OUTDIR
set -euo pipefail
out="$1"
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o bench --output-format csv -- \
  python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > "$out/trace_bench.json" 2> "$out/trace_bench.err"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o p --output-format csv -- \
  python3 tools/kernel_sweep.py 400 0 > "$out/fetch.log" 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o p --output-format csv -- \
  python3 tools/kernel_sweep.py 400 0 > "$out/write.log" 2>&1
