#!/usr/bin/env bash
# Same-box A/B of config 3 (refracted forward): default library vs variants/old.so (bench + kernel stats)
set -o pipefail
o=gpurun_out/ab3; mkdir -p $o
export TMPDIR=/tmp
for v in new old new2; do
  lib=""; [ "$v" = old ] && lib=variants/old.so
  TVAM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/$v -o k --output-format csv -- python3 bench.py --config 3 --steps 10 --cpu-baseline off > $o/$v.json 2> $o/$v.err || exit 1
done
