#!/usr/bin/env bash
# A/B of libtvam builds on config 2: for each NAME, tools/proj_ab.py under TVAM_LIB=_variants/libtvam_NAME.so
# (NAME "head" = the in-tree drtvam_amd/libtvam.so); extra proj_ab variants via $VARIANTS.
# usage (on the GPU box): tools/lib_ab.sh OUTDIR NAME...
set -eo pipefail
out="$1"; shift
mkdir -p "$out"
for rep in 1 2; do
  for name in "$@"; do
    lib="_variants/libtvam_$name.so"; [ "$name" = head ] && lib="drtvam_amd/libtvam.so"
    echo "== $name (rep $rep)"
    TVAM_LIB="$lib" TVAM_EXPERIMENTAL=1 timeout -k 10 240 python3 -u tools/proj_ab.py 400 ${VARIANTS:-""} \
      | sed "s/^{/{\"lib\": \"$name\", \"rep\": $rep, /" | tee -a "$out/proj_ab.jsonl"
  done
done
