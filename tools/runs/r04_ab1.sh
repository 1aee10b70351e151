#!/usr/bin/env bash
# Round 4 A/B: paired-voxel forward (config 2) and counting-sort brick bins (config 4), then the
# parity tests these touch.  usage: tools/runs/r04_ab1.sh OUT
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 300 python tools/fwd_px_ab.py 400 "TVAM_FWD_PX=1" "TVAM_FWD_PX=2" "TVAM_FWD_PX=2 TVAM_PLANAR_FWD_Z=24" \
  "TVAM_FWD_PX=1 TVAM_PLANAR_FWD_Z=24" "TVAM_FWD_PX=2 TVAM_PLANAR_FWD_Z=16" > "$o/fwd_ab.jsonl" 2> "$o/fwd_ab.err"
timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --cpu-baseline off > "$o/c4_csort.json" 2> "$o/c4_csort.err"
TVAM_BIN_SORT=1 timeout -k 10 400 python bench.py --config 4 --steps 3 --warmup 1 --cpu-baseline off > "$o/c4_radix.json" 2> "$o/c4_radix.err"
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scattering.py \
  tests/test_gpu_bin_chunks.py tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_active_set.py \
  tests/test_gpu_distributed.py tests/test_gpu_bench.py > "$o/tests.log" 2>&1
