set -euo pipefail
o=gpurun_out/r04/px; mkdir -p $o
timeout -k 10 300 python tools/fwd_px_ab.py 400 "TVAM_FWD_PX=1" "TVAM_FWD_PX=2" "TVAM_FWD_PX=2 TVAM_PLANAR_FWD_Z=24" "TVAM_FWD_PX=1 TVAM_PLANAR_FWD_Z=24" "TVAM_FWD_PX=2 TVAM_PLANAR_FWD_Z=16" > $o/ab.jsonl 2> $o/ab.err
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_active_set.py tests/test_gpu_distributed.py tests/test_gpu_bench.py > $o/tests.log 2>&1
