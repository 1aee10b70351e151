#!/usr/bin/env bash
# Round-5 record, part B: counters of configs 4 and 5 (tools/pmc_bench.sh).  usage: tools/runs/r05_final_b.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
tools/pmc_bench.sh "$o/pmc_c4" 4
tools/pmc_bench.sh "$o/pmc_c5" 5 800
