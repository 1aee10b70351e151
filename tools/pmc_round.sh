#!/usr/bin/env bash
# SQ / TCC counters of the config-2 forward and adjoint kernels (tools/kernel_sweep.py 400 0),
# one rocprofv3 --pmc pass per counter set (never combined with tracing), plus a kernel-trace
# --stats pass of the same program for the kernels' durations.
# usage (GPU box, repo root): tools/pmc_round.sh OUTDIR [kernel_sweep args]
set -euo pipefail
out="$1"; shift
args="${*:-400 0}"
export TMPDIR=/tmp
mkdir -p "$out"
sets=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
  "WRITE_SIZE"
)
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set -d "$out/p$i" -o p --output-format csv -- \
    python3 tools/kernel_sweep.py $args > "$out/p$i.log" 2>&1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/trace" -o k --output-format csv -- \
  python3 tools/kernel_sweep.py $args > "$out/trace.log" 2>&1
