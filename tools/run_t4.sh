set -eo pipefail
o=gpurun_out/r06/t4; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o k --output-format csv -- python3 bench.py --config 2 --emulate 3/8 --shard slab --steps 20 --warmup 2 > $o/slab3.json 2> $o/slab3.err
