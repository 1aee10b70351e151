# A/B of the speculative L-BFGS update on one box: config-2 bench lines with FusedLinearLBFGS.speculate
# on and off, alternating.  tools/spec_ab.sh OUT N
set -eo pipefail
o=$1; n=${2:-3}; mkdir -p $o
for i in $(seq 1 $n); do
  for s in True False; do
    timeout -k 10 240 python3 -c "
import sys, runpy
import drtvam_amd.lbfgs as L
L.FusedLinearLBFGS.speculate = $s
sys.argv = ['bench.py', '--cpu-baseline', 'off']
runpy.run_path('bench.py', run_name='__main__')" | sed "s/^{/{\"speculate\": $s, /" >> $o/spec_ab.jsonl 2>> $o/err.log
  done
done
