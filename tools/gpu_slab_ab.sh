#!/usr/bin/env bash
# Thin-slab adjoint A/B: rank 3 of 8 and rank 0 of 4 (z-slab emulation) under adjoint splits / workgroup sizes
set -o pipefail
o=gpurun_out/slab_ab; mkdir -p $o
for cfg in "TVAM_DEFAULT=1" "TVAM_ADJ_SPLIT=1" "TVAM_ADJ_SPLIT=2" "TVAM_ADJ_SPLIT=4" "TVAM_ADJ_SPLIT=16" "TVAM_ADJ_NT=512"; do
  for rw in 3/8 0/4; do
    env $cfg timeout -k 10 120 python bench.py --emulate $rw --steps 20 --warmup 3 2>> $o/err.log | sed "s/^{/{\"env\": \"$cfg\", /" >> $o/emulate.jsonl || exit 1
  done
done
