# kernel traces of the config-2 bench with the speculative L-BFGS update on and off, and their idle gaps
set -eo pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp
for s in True False; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $o/t$s -o k --output-format csv -- python3 -c "
import sys, runpy
import drtvam_amd.lbfgs as L
L.FusedLinearLBFGS.speculate = $s
sys.argv = ['bench.py', '--cpu-baseline', 'off', '--steps', '20']
runpy.run_path('bench.py', run_name='__main__')" > $o/bench_$s.json 2> $o/err_$s.log
  python3 tools/trace_gaps.py $(find $o/t$s -name '*kernel_trace.csv' | head -1) 100 > $o/gaps_$s.txt
  find $o/t$s -name '*kernel_trace.csv' -delete
done
