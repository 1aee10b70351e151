#!/usr/bin/env bash
# Round 4: voxel-driven forward grid / tail variants on config 2 (tools/proj_ab.py).  usage: tools/runs/r04_ab5.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 python tools/proj_ab.py 400 "" "TVAM_FWD_PARTS=2" "TVAM_FWD_PARTS=3" "TVAM_XCD_REMAP=0" \
  "TVAM_FWD_PX=2 TVAM_PLANAR_FWD_Z=16" "TVAM_PLANAR_FWD_Z=28" > "$o/proj_ab.jsonl" 2> "$o/proj_ab.err"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > "$o/tests.log" 2>&1
