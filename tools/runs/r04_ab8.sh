#!/usr/bin/env bash
# Round 4: closed-form brick counts in the record writer + the device-side L-BFGS recursion
# (current tree) against HEAD (_variants/head: HEAD's sources with its own build).
# usage: tools/runs/r04_ab8.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
c2="--steps 20 --warmup 2 --cpu-baseline off"
c4="--config 4 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off"
timeout -k 10 150 python bench.py $c2 > "$o/c2_new.json" 2> "$o/c2_new.err"
(cd _variants/head && timeout -k 10 150 python bench.py $c2) > "$o/c2_head.json" 2> "$o/c2_head.err"
timeout -k 10 240 python bench.py $c4 > "$o/c4_new.json" 2> "$o/c4_new.err"
(cd _variants/head && timeout -k 10 240 python bench.py $c4) > "$o/c4_head.json" 2> "$o/c4_head.err"
timeout -k 10 150 python bench.py $c2 > "$o/c2_new2.json" 2> "$o/c2_new2.err"
(cd _variants/head && timeout -k 10 150 python bench.py $c2) > "$o/c2_head2.json" 2> "$o/c2_head2.err"
