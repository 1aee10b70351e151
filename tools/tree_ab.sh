# A/B of two source trees on one box: the config-2 bench line of _variants/base (a `git archive` of an
# earlier commit with its own libtvam.so) and of this tree, alternating.  tools/tree_ab.sh OUT N
set -eo pipefail
o=$(realpath -m $1); n=${2:-3}; mkdir -p $o
for i in $(seq 1 $n); do
  (cd _variants/base && timeout -k 10 240 python3 bench.py --cpu-baseline off | sed 's/^{/{"tree": "base", /' >> $o/tree_ab.jsonl 2>> $o/err.log)
  timeout -k 10 240 python3 bench.py --cpu-baseline off | sed 's/^{/{"tree": "head", /' >> $o/tree_ab.jsonl 2>> $o/err.log
done
