#!/usr/bin/env bash
# Counters of one BASELINE config's bench iteration for the committed roofline summaries
# (tools/roofline_summary.py -> profiles/r06/roofline_config<K>.json, read by bench.py; tools/pmc_final.sh):
# one rocprofv3 --pmc pass per counter set (never combined with tracing, each within the
# per-block limits), then a --kernel-trace --stats pass of the same command.
# usage (GPU box, repo root): tools/pmc_bench.sh OUT CONFIG [N]
set -euo pipefail
out="$1"; c="$2"; n="${3:-400}"
export TMPDIR=/tmp
mkdir -p "$out"
# --slab-bands 1: the planar configs' kernels as full-film launches (the summaries' per-launch bytes)
cmd=(python3 bench.py --config "$c" --n "$n" --steps 1 --warmup 0 --prewarm 0 --cpu-baseline off --slab-bands 1)
echo "${cmd[*]}" > "$out/command.txt"
python3 -c "import bench; print(bench.csrc_digest())" > "$out/csrc_sha16.txt"
sets=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
  "WRITE_SIZE"
)
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $set -d "$out/p$i" -o p --output-format csv -- "${cmd[@]}" > "$out/p$i.log" 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o k --output-format csv -- "${cmd[@]}" > "$out/trace.log" 2>&1
