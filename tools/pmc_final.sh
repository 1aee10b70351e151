#!/usr/bin/env bash
# Counter passes of one BASELINE config (tools/pmc_bench.sh) summarised on the box into the committed
# roofline summary (tools/roofline_summary.py) and the same command's kernel stats; the raw
# per-dispatch CSVs are deleted (a scattering config's run to run exceeds gpurun's copy-back limit).
# usage (GPU box, repo root): tools/pmc_final.sh OUT CONFIG "KERNEL PREFIX" BOUND MIN_BYTES
set -euo pipefail
out="$1"; c="$2"; kern="$3"; bound="$4"; minb="$5"
n=400; [ "$c" = 5 ] && n=800
bash tools/pmc_bench.sh "$out/c$c" "$c" "$n"
python3 tools/roofline_summary.py "$out/c$c" "$c" "$kern" "$bound" "$out/roofline_config$c.json" "$minb"
cp "$out/c$c/trace/k_kernel_stats.csv" "$out/config${c}_kernel_stats.csv"
find "$out/c$c" -name '*.csv' -delete
echo "config $c summarised" >&2
