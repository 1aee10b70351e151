#!/bin/bash
# Round-5 record: config 2's angle-shard rank 0 of 8 (bench.py --emulate 0/8 --shard angle) with
# the list adjoint at 16 and 8 slices per workgroup and with the tile adjoint (no visit lists).
# Results: profiles/r05/ab_angle_shard_adjoint/.
set -e
o=gpurun_out/r05/emu_angle2_ab
mkdir -p "$o"
export TVAM_EXPERIMENTAL=1
for v in "TVAM_ADJL_Z=16" "TVAM_ADJL_Z=8" "TVAM_ADJ_LISTS=0"; do
    env $v timeout -k 10 120 python bench.py --emulate 0/8 --shard angle --steps 10 --warmup 2 \
        --cpu-baseline off > "$o/$v.json" 2> "$o/$v.err"
done
