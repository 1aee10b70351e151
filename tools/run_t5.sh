set -eo pipefail
o=gpurun_out/r06/t5; mkdir -p $o
for v in "" "TVAM_ADJL_Z=16" "TVAM_FWD_PARTS=2" "TVAM_FWD_PARTS=3" "TVAM_FWD_PARTS=6" "TVAM_PLANAR_FWD_Z=24" "TVAM_PLANAR_FWD_Z=28"; do
  for r in 3 0; do
    env $v TVAM_EXPERIMENTAL=1 timeout -k 10 180 python bench.py --config 2 --emulate $r/8 --shard slab --steps 20 --warmup 2 2>> $o/err.log | sed "s|^{|{\"knob\": \"$v\", |" >> $o/knobs.jsonl
  done
done
