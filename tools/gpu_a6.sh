#!/usr/bin/env bash
# Config-4 adjoint brick-march A/B on a 40-angle shard: default, no partial stores (debug), 512-thread workgroups
set -o pipefail
o=gpurun_out/a6; mkdir -p $o
export TMPDIR=/tmp
run() {  # name, then env assignments
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/$name -o k --output-format csv -- \
    python3 tools/profile_jitter.py 4 400 40 2 > $o/$name.log 2>&1
}
run default TVAM_BIN_NT=1024 || exit 1
run nopart TVAM_LIB=variants/nopart.so || exit 1
run nt512 TVAM_BIN_NT=512
