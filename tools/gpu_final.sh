#!/usr/bin/env bash
# Final record (GPU box): the whole -m gpu suite, smoke, config 2 bench + rocprofv3 stats, then the z-slab
# scaling emulation.  usage: tools/gpu_final.sh OUT
set -o pipefail
o="$1"; mkdir -p "$o"
bash tools/round_final.sh "$o" || exit 1
bash tools/scale_emulate.sh "$o/slab"
