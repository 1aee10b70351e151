#!/usr/bin/env bash
# rocprofv3 kernel stats of one config-5 iteration (GPU box, repo root): tools/profile_config5.sh OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/trace5 -o c5 --output-format csv -- \
  python3 bench.py --config 5 --n 800 --steps 1 --warmup 1 --cpu-baseline off > $o/c5_bench.json 2> $o/c5_bench.err
