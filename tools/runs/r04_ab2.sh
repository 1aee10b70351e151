#!/usr/bin/env bash
# Round 4 A/B benches: projection variants of config 2 (tools/proj_ab.py), configs 2/4/5 bench lines
# with the current defaults and with the previous paths (TVAM_BIN_SORT=1 and the no-prefetch tile
# build), then the parity tests of the changed kernels.  usage: tools/runs/r04_ab2.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 240 python tools/proj_ab.py 400 "TVAM_FWD_PX=1 TVAM_ADJ_PAIR=0" "" "TVAM_PLANAR_FWD_Z=24" \
  "TVAM_ADJ_PAIR=0" "TVAM_PLANAR_ADJ_Z=16" "TVAM_PLANAR_ADJ_Z=16 tile=32" > "$o/proj_ab.jsonl" 2> "$o/proj_ab.err"
timeout -k 10 200 python bench.py --cpu-baseline off > "$o/c2.json" 2> "$o/c2.err"
timeout -k 10 200 python bench.py --config 4 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c4.json" 2> "$o/c4.err"
TVAM_BIN_SORT=1 TVAM_LIB=$PWD/_variants/libtvam_nopf.so timeout -k 10 200 python bench.py --config 4 --steps 2 --warmup 1 \
  --prewarm 0 --cpu-baseline off > "$o/c4_old.json" 2> "$o/c4_old.err"
timeout -k 10 200 python bench.py --config 5 --n 800 --steps 2 --warmup 1 --prewarm 0 --cpu-baseline off > "$o/c5.json" 2> "$o/c5.err"
TVAM_LIB=$PWD/_variants/libtvam_nopf.so timeout -k 10 200 python bench.py --config 5 --n 800 --steps 2 --warmup 1 \
  --prewarm 0 --cpu-baseline off > "$o/c5_nopf.json" 2> "$o/c5_nopf.err"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$o/tests.log" 2>&1
