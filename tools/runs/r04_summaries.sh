#!/usr/bin/env bash
# Round-4 roofline summaries from the pmc_bench directories of tools/runs/r04_final_{a,b}.sh (run on
# this machine after the GPU calls): profiles/r04/roofline_config<K>.json + the kernel stats of
# the same command (profiles/r04/pmc/config<K>_kernel_stats.csv, checked by tests/test_bench_roofline.py).
# usage: tools/runs/r04_summaries.sh CONFIG PMC_DIR
set -euo pipefail
c="$1"; src="$2"
mkdir -p profiles/r04/pmc
case "$c" in
  2) k="void tvam_fwd_planar_kernel<32, 2, false, 1, 2, true, false, 1>"; b=lds; m=556000000 ;;
  3) k="void tvam_fwd_planar_kernel<32, 2, false, 2, 2, true, true, 1>"; b=lds; m=570000000 ;;
  # config 4: each entry's 48-byte record and 4-byte slot read once (519.3 M entries per chunk
  # launch: 11.94e9 per pass / 23 chunks) + the dose read and written once
  4) k="void (anonymous namespace)::tvam_bin_march_kernel<0, 1024, false>"; b=hbm; m=27500000000 ;;
  5) k="void tvam_tile_kernel<0, true>"; b=valu; m=86000000000 ;;
esac
python tools/roofline_summary.py "$src" "$c" "$k" "$b" "profiles/r04/roofline_config$c.json" "$m"
cp "$src/trace/k_kernel_stats.csv" "profiles/r04/pmc/config${c}_kernel_stats.csv"
