#!/usr/bin/env bash
# Kernel stats of the BASELINE configs 3-5 (bench.py --config N), one rocprofv3
# kernel-trace pass each (GPU box, repo root): tools/profile_configs.sh OUTDIR
set -euo pipefail
out="$1"
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/c3" -o c3 --output-format csv -- \
  python3 bench.py --config 3 --steps 5 --warmup 2 --cpu-baseline off > "$out/c3_bench.json" 2> "$out/c3_bench.err"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/c4" -o c4 --output-format csv -- \
  python3 bench.py --config 4 --steps 1 --warmup 1 --cpu-baseline off > "$out/c4_bench.json" 2> "$out/c4_bench.err"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out/c5" -o c5 --output-format csv -- \
  python3 bench.py --config 5 --n 800 --steps 1 --warmup 1 --cpu-baseline off > "$out/c5_bench.json" 2> "$out/c5_bench.err"
