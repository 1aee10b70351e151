#!/bin/bash
# Round-5 record: counters of config 2's angle-shard rank 0 of 8 (one emulated iteration), for
# the list adjoint's poor angle scaling.  Same counter sets as
# tools/pmc_bench.sh, one rocprofv3 --pmc pass each.
set -euo pipefail
out=gpurun_out/r05/angle_pmc
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 bench.py --emulate 0/8 --shard angle --steps 1 --warmup 0 --cpu-baseline off)
sets=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
  "WRITE_SIZE"
)
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set -d "$out/p$i" -o p --output-format csv -- "${cmd[@]}" > "$out/p$i.log" 2>&1
done
