set -eo pipefail
o=gpurun_out/r06/z48; mkdir -p $o
for rep in 1 2; do
for lib in head z48; do
  L=_variants/libtvam_$lib.so; [ $lib = head ] && L=drtvam_amd/libtvam.so
  for r in 1 3 7; do
    TVAM_LIB=$L timeout -k 10 180 python bench.py --config 2 --emulate $r/8 --shard slab --steps 20 --warmup 2 2>> $o/err.log | sed "s|^{|{\"lib\": \"$lib\", |" >> $o/emu.jsonl
  done
done
done
