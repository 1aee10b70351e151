#!/usr/bin/env bash
# Counter passes (one rocprofv3 --pmc run per set, never with tracing) + a kernel-trace --stats pass of
# tools/profile_jitter.py.  usage (GPU box, repo root): tools/pmc_jitter.sh OUTDIR CONFIG N ANGLES
set -euo pipefail
out="$1"; shift
export TMPDIR=/tmp
mkdir -p "$out"
sets=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $set -d "$out/p$i" -o p --output-format csv -- \
    python3 tools/profile_jitter.py "$@" > "$out/p$i.log" 2>&1
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$out/trace" -o k --output-format csv -- \
  python3 tools/profile_jitter.py "$@" > "$out/trace.log" 2>&1
