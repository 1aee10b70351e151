#!/usr/bin/env bash
# Collects SQ counters for tools/kernel_sweep.py in separate rocprofv3 passes
# (one counter set per pass; never combined with tracing).
# usage (on the GPU box, from the repo root): tools/pmc.sh OUTDIR [sweep args...]
# PMC_SETS (optional): counter sets separated by ';'
set -euo pipefail
out="$1"; shift
export TMPDIR=/tmp
mkdir -p "$out"
default="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
IFS=';' read -ra sets <<< "${PMC_SETS:-$default}"
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -d "$out/p$i" -o p --output-format csv -- python3 tools/kernel_sweep.py "$@" > "$out/p$i.log" 2>&1
done
