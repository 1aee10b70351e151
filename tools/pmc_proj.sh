#!/usr/bin/env bash
# Counters of tools/proj_ab.py projection variants (config 2), one rocprofv3 --pmc pass per set
# (never combined with tracing), summarised per kernel by tools/pmc_summary.py.
# usage (GPU box, repo root): tools/pmc_proj.sh OUT "variant" ...
set -o pipefail
out="$1"; shift
export TMPDIR=/tmp
mkdir -p "$out"
sets=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
v=0
for var in "$@"; do
  v=$((v+1))
  i=0; mkdir -p "$out/v$v"
  for set in "${sets[@]}"; do
    i=$((i+1))
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $set -d "$out/v$v/p$i" -o p --output-format csv -- python3 tools/proj_ab.py 400 "$var" > "$out/v$v/p$i.log" 2>&1 || exit 1
  done
  echo "variant $v: $var" >> "$out/summary.txt"
  python3 tools/pmc_summary.py "$out/v$v" >> "$out/summary.txt"
done
