#!/usr/bin/env bash
# Round 4: the whole -m gpu suite on the current build, then tools/runs/r04_ab9.sh.  usage: tools/runs/r04_tests2.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > "$o/gpu_tests.log" 2>&1
tools/runs/r04_ab9.sh "$o/ab9"
