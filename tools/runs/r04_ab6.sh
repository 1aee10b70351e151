#!/usr/bin/env bash
# Round 4: packed crossing step + two visits per loop trip in the tile march and the planar adjoint
# (current build) against the previous build (_variants/libtvam_head.so).  usage: tools/runs/r04_ab6.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
TVAM_LIB=$PWD/_variants/libtvam_head.so timeout -k 10 200 python tools/proj_ab.py 400 "" > "$o/proj_head.jsonl" 2> "$o/proj_head.err"
timeout -k 10 200 python tools/proj_ab.py 400 "" > "$o/proj_new.jsonl" 2> "$o/proj_new.err"
TVAM_LIB=$PWD/_variants/libtvam_head.so timeout -k 10 200 python tools/proj_ab.py 400 "" > "$o/proj_head2.jsonl" 2> "$o/proj_head2.err"
timeout -k 10 200 python tools/proj_ab.py 400 "" > "$o/proj_new2.jsonl" 2> "$o/proj_new2.err"
timeout -k 10 200 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c5_new.json" 2> "$o/c5_new.err"
TVAM_LIB=$PWD/_variants/libtvam_head.so timeout -k 10 200 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --prewarm 0 \
  --cpu-baseline off > "$o/c5_head.json" 2> "$o/c5_head.err"
timeout -k 10 200 python bench.py --config 4 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c4_new.json" 2> "$o/c4_new.err"
TVAM_LIB=$PWD/_variants/libtvam_head.so timeout -k 10 200 python bench.py --config 4 --steps 2 --warmup 1 --prewarm 0 \
  --cpu-baseline off > "$o/c4_head.json" 2> "$o/c4_head.err"
