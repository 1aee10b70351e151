#!/usr/bin/env bash
# Round 5: the whole -m gpu suite and smoke() on the final committed tree.  usage: tools/runs/r05_final_tests.sh OUT
set -euo pipefail
o="$(realpath -m "$1")"; mkdir -p "$o"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  > "$o/gpu_tests.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$o/smoke.log" 2>&1
