# config-2 bench line repeated on one box (box-to-box spread check): tools/bench_repeat.sh OUT N
set -eo pipefail
o=$1; n=${2:-3}; mkdir -p $o
for i in $(seq 1 $n); do
  timeout -k 10 240 python3 bench.py --cpu-baseline off >> $o/bench_repeat.jsonl 2>> $o/err.log
done
