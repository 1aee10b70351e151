#!/usr/bin/env bash
# Round 4: (1) the voxel-driven jittered forward prototype (tools/proto_vox_jitter.hip: small
# check against a CPU clip, then config 5's size) next to config 5's production forward on the
# same box; (2) launch-geometry sweep of the L-BFGS vector passes (tools/vec_sweep.py).
# usage: tools/runs/r04_ab9.sh OUT   (tools/build/proto_vox_jitter prebuilt)
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 120 tools/build/proto_vox_jitter 64 6 4 check > "$o/proto_check.jsonl" 2> "$o/proto_check.err"
timeout -k 10 240 tools/build/proto_vox_jitter 800 800 4 > "$o/proto_800.jsonl" 2> "$o/proto_800.err"
timeout -k 10 240 python bench.py --config 5 --n 800 --steps 1 --warmup 1 --prewarm 0 --cpu-baseline off \
  > "$o/c5.json" 2> "$o/c5.err"
for hg in 768 1536 2048; do
  for dg in 1024 2048 4096; do
    TVAM_VEC_HGRID=$hg TVAM_VEC_DGRID=$dg timeout -k 10 120 python tools/vec_sweep.py >> "$o/vec_sweep.jsonl" 2>> "$o/vec_sweep.err"
  done
done
