#!/usr/bin/env bash
# Round-end record of the final build: counters of configs 2-5 (summarised on the box), the -m gpu
# suite, smoke, the config-2 bench line (+ rocprofv3 stats), configs 3-5 bench lines, all 8 ranks of
# both config-2 splits.  usage (GPU box, repo root): tools/final_all.sh OUT PART   (PART: pmc | run)
set -euo pipefail
o=$1; part=$2; mkdir -p $o
if [ "$part" = pmc ]; then
  bash tools/pmc_final.sh $o/pmc 2 "void tvam_fwd_planar_kernel<52, 2, false, 1, 2, true, false, true>" lds 556000000
  bash tools/pmc_final.sh $o/pmc 3 "void tvam_fwd_planar_kernel<32, 2, false, 1, 2, true, true, true>" lds 570000000
  bash tools/pmc_final.sh $o/pmc 4 "void (anonymous namespace)::tvam_bin_march_kernel<0, 1024, false>" hbm 27500000000
  bash tools/pmc_final.sh $o/pmc 5 "void tvam_tile_kernel<0, true>" valu 86000000000
else
  bash tools/round_final.sh $o
  rm -f $o/prof/k_kernel_trace.csv
  bash tools/final_configs.sh $o
  bash tools/emulate8.sh $o slab angle
fi
