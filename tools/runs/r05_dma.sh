#!/usr/bin/env bash
# Forward LDS-DMA staging A/B on config 2 (tools/proj_ab.py, interleaved libraries), then the planar
# parity tests on the default library.  usage: tools/runs/r05_dma.sh OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in base dma256 cur; do
    lib=tools/build/libtvam_$v.so; [ $v = cur ] && lib=drtvam_amd/libtvam.so
    echo "{\"lib\": \"$v\"}" >> $o/ab.jsonl
    TVAM_LIB=$lib timeout -k 10 200 python -u tools/proj_ab.py 400 >> $o/ab.jsonl 2>>$o/err.log || exit 1
  done
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_slice_bin.py tests/test_gpu_baseline_sizes.py -k "not config4 and not config5" > $o/tests.log 2>&1 || exit 1
