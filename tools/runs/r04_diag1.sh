#!/usr/bin/env bash
# Round 4: the one-angle config-4 calls step by step: default build, counting-sort bins, no-prefetch build
set -uo pipefail
o="$1"; mkdir -p "$o"
timeout -k 10 120 python -u tools/diag_one_angle.py 4 > "$o/default.log" 2>&1; rc=$?; echo "rc=$rc" >> "$o/default.log"
[ $rc -eq 0 ] || exit $rc
TVAM_BIN_SORT=0 timeout -k 10 120 python -u tools/diag_one_angle.py 4 > "$o/csort.log" 2>&1; rc=$?; echo "rc=$rc" >> "$o/csort.log"
[ $rc -eq 0 ] || exit $rc
TVAM_LIB=$PWD/_variants/libtvam_nopf.so timeout -k 10 120 python -u tools/diag_one_angle.py 4 > "$o/nopf.log" 2>&1; rc=$?; echo "rc=$rc" >> "$o/nopf.log"
exit $rc
