#!/usr/bin/env bash
# Round 4: the pattern-binning transpose prototype (tools/proto_slice_bin.hip, prebuilt).  usage: tools/runs/r04_proto_bin.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
timeout -k 10 120 tools/build/proto_slice_bin > "$o/proto_slice_bin.jsonl" 2> "$o/proto_slice_bin.err"
timeout -k 10 120 tools/build/proto_slice_bin 400 800 800 >> "$o/proto_slice_bin.jsonl" 2>> "$o/proto_slice_bin.err"
