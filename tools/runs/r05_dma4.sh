#!/usr/bin/env bash
# LDS-DMA staging as a per-plan choice: config 2 A/B vs register staging, the 8-rank slab emulation
# (50-slice slabs, Z = 52), then the planar / refracted / slab GPU tests.  usage: tools/runs/r05_dma4.sh OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for v in base cur; do
  lib=tools/build/libtvam_$v.so; [ $v = cur ] && lib=drtvam_amd/libtvam.so
  echo "{\"lib\": \"$v\"}" >> $o/ab2.jsonl
  TVAM_LIB=$lib timeout -k 10 200 python -u tools/proj_ab.py 400 >> $o/ab2.jsonl 2>>$o/err.log || exit 1
  TVAM_LIB=$lib timeout -k 10 200 python bench.py --emulate 3/8 --shard slab --steps 10 --warmup 2 --cpu-baseline off >> $o/emu_$v.jsonl 2>>$o/err.log || exit 1
done
timeout -k 10 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cylindrical.py tests/test_gpu_parity.py tests/test_gpu_slice_bin.py tests/test_gpu_distributed.py tests/test_gpu_pipeline.py > $o/tests.log 2>&1 || exit 1
