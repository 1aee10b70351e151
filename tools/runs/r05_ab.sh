#!/usr/bin/env bash
# round-5 A/B on the GPU box: projection variants (tools/proj_ab.py), then selected GPU tests.
# usage: tools/runs/r05_ab.sh OUT "variant" ... -- [pytest args]
set -o pipefail
o=$1; shift; mkdir -p $o
vars=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/proj_ab.py 400 "${vars[@]}" > $o/proj_ab.jsonl 2> $o/proj_ab.err || exit 1
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $o/tests.log 2>&1 || exit 1
fi
