#!/usr/bin/env bash
# Forward LDS-DMA staging (refracted records too) vs register staging (tools/build/libtvam_base.so):
# config 2 (proj_ab) and config 3 (profile_jitter, all 400 angles), interleaved; then the refracted
# and planar parity tests on the default library.  usage: tools/runs/r05_dma3.sh OUT
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in base cur; do
    lib=tools/build/libtvam_$v.so; [ $v = cur ] && lib=drtvam_amd/libtvam.so
    echo "{\"lib\": \"$v\"}" >> $o/ab2.jsonl
    TVAM_LIB=$lib timeout -k 10 200 python -u tools/proj_ab.py 400 >> $o/ab2.jsonl 2>>$o/err.log || exit 1
    echo "lib $v" >> $o/c3.log
    TVAM_LIB=$lib timeout -k 10 200 python -u tools/profile_jitter.py 3 400 200 3 >> $o/c3.log 2>&1 || exit 1
  done
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cylindrical.py tests/test_gpu_parity.py > $o/tests.log 2>&1 || exit 1
