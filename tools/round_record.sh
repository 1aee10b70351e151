#!/usr/bin/env bash
# Round record (GPU box, repo root): the whole -m gpu suite, smoke(), the default bench line (config 2),
# rocprofv3 kernel stats of the same bench command, then bench lines of configs 3-5.
# usage: tools/round_record.sh OUT
set -o pipefail
o="$1"; mkdir -p "$o"
bash tools/round_final.sh "$o" || exit 1
bash tools/configs_bench.sh "$o"
