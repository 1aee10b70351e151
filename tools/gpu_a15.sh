#!/usr/bin/env bash
# Adjoint split cap 4: slab / distributed / parity suites, then the z-slab scaling emulation
set -o pipefail
o=gpurun_out/a15; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_adj_quadrants.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1 || exit 1
bash tools/scale_emulate.sh $o/slab
