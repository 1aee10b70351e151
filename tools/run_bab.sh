# bench.py config 2 under alternative libtvam builds (TVAM_LIB), interleaved: usage tools/run_bab.sh OUT NAME...
set -eo pipefail
o=$1; shift; mkdir -p $o
for rep in 1 2; do
  for lib in "$@"; do
    TVAM_LIB=_variants/libtvam_$lib.so timeout -k 10 240 python3 bench.py --cpu-baseline off 2>> $o/err.log | sed "s|^{|{\"lib\": \"$lib\", |" >> $o/bench.jsonl
  done
done
