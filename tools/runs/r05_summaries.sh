#!/usr/bin/env bash
# Round-5 roofline summaries (profiles/r05) from the final counter runs (tools/runs/r05_final_a.sh, _b.sh).
set -euo pipefail
A=${1:-gpurun_out/r05/final_a}; B=${2:-gpurun_out/r05/final_b}; P=profiles/r05
mkdir -p $P/pmc $P/secondary
python3 tools/roofline_summary.py $A/pmc_c2 2 "void tvam_fwd_planar_kernel<52, 2, false, 1, 2, true, false, true>" lds $P/roofline_config2.json 556000000 > /dev/null
python3 tools/roofline_summary.py $A/pmc_c3 3 "void tvam_fwd_planar_kernel<32, 2, false, 1, 2, true, true, true>" lds $P/roofline_config3.json 570000000 > /dev/null
python3 tools/roofline_summary.py $A/pmc_c2 2 "void tvam_adjl_kernel<16, 1024, 1, 8>" lds $P/secondary/roofline_config2_adjoint.json > /dev/null
python3 tools/roofline_summary.py $B/pmc_c4 4 "void (anonymous namespace)::tvam_bin_march_kernel<0, 1024, false>" hbm $P/roofline_config4.json 27500000000 > /dev/null
python3 tools/roofline_summary.py $B/pmc_c5 5 "void tvam_tile_kernel<0, true>" valu $P/roofline_config5.json 86000000000 > /dev/null
python3 tools/roofline_summary.py $B/pmc_c4 4 "void (anonymous namespace)::tvam_bin_march_kernel<2, 1024, false>" hbm $P/secondary/roofline_config4_adjoint_march.json > /dev/null
python3 tools/roofline_summary.py $B/pmc_c5 5 "void tvam_tile_kernel<1, true>" valu $P/secondary/roofline_config5_adjoint.json > /dev/null
for c in 2 3; do cp "$(find $A/pmc_c$c/trace -name '*kernel_stats.csv')" $P/pmc/config${c}_kernel_stats.csv; done
for c in 4 5; do cp "$(find $B/pmc_c$c/trace -name '*kernel_stats.csv')" $P/pmc/config${c}_kernel_stats.csv; done
