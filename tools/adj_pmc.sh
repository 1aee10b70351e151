#!/usr/bin/env bash
# SQ counters of the config-2 planar adjoint per plan-time variant (tools/adj_variants.py), one
# rocprofv3 --pmc pass per variant.  usage (GPU box): tools/adj_pmc.sh OUT "K=V,.." "K=V" ...
set -euo pipefail
out="$1"; shift; mkdir -p "$out"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  echo "$v" > "$out/v$i.txt"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$out/v$i" -o p --output-format csv -- \
    python3 tools/adj_variants.py "$v" > "$out/v$i.log" 2>&1
done
