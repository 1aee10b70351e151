#!/usr/bin/env bash
# counters of config 5's tile kernels on a 100-angle shard, slot orders 2 (default) and 0
set -o pipefail
o=$1; mkdir -p $o
export TMPDIR=/tmp TVAM_EXPERIMENTAL=1
for ss in 2 0; do
  export TVAM_SLOT_SORT=$ss; mkdir -p $o/ss$ss
  timeout -k 10 300 python3 tools/profile_jitter.py 5 800 100 2 > $o/time_ss$ss.log 2>&1 || exit 1
  i=0
  for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM"; do
    i=$((i+1))
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $set -d $o/ss$ss/p$i -o p --output-format csv -- python3 tools/profile_jitter.py 5 800 100 > $o/ss$ss/p$i.log 2>&1 || exit 1
  done
  echo "slot sort $ss" >> $o/summary.txt
  python3 tools/pmc_summary.py $o/ss$ss >> $o/summary.txt
done
