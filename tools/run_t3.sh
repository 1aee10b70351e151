set -eo pipefail
o=gpurun_out/r06/t3; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_zero_tiles.py tests/test_gpu_baseline_sizes.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $o/tests.log 2>&1
timeout -k 10 240 python3 -u tools/proj_ab.py 400 > $o/proj_ab.jsonl 2>> $o/proj_ab.err
bash tools/emulate8.sh $o angle
