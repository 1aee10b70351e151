#!/usr/bin/env bash
# Forward depth re-priced for the LDS-DMA staging (Z = 52 on 400-slice films): config 2 A/B against
# Z = 32, the bench line, then the planar / pipeline / distributed GPU tests.  usage: OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
TVAM_EXPERIMENTAL=1 timeout -k 10 300 python -u tools/proj_ab.py 400 "" "TVAM_PLANAR_FWD_Z=32" "" "TVAM_PLANAR_FWD_Z=32" > $o/proj_ab.jsonl 2> $o/proj_ab.err || exit 1
timeout -k 10 300 python bench.py --cpu-baseline off > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_distributed.py tests/test_gpu_rccl.py tests/test_gpu_slice_bin.py tests/test_gpu_kernel_time.py tests/test_gpu_baseline_sizes.py tests/test_gpu_cylindrical.py > $o/tests.log 2>&1 || exit 1
