#!/usr/bin/env bash
# Per-ray tile kernels under each TVAM_SLOT_SORT mode: one rocprofv3 --pmc pass (VALU issue and
# lane utilisation counters) of tools/profile_jitter.py per mode.  usage: tools/slot_sort_ab.sh OUT CONFIG N ANGLES
set -euo pipefail
out="$1"; shift; mkdir -p "$out"
export TMPDIR=/tmp
for m in 0 1 2; do
  TVAM_SLOT_SORT=$m timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$out/m$m" -o p --output-format csv -- \
    python3 tools/profile_jitter.py "$@" > "$out/m$m.log" 2>&1
done
