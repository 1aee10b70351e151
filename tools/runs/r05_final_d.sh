#!/usr/bin/env bash
# Round-5 record, part D: the 8-rank angle-shard emulations of configs 4 and 5 (tools/emulate_angle8.sh).
set -euo pipefail
o="$1"; mkdir -p "$o"
export TMPDIR=/tmp
tools/emulate_angle8.sh "$o/emulate_angle8" 4 5
