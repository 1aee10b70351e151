set -o pipefail
o=gpurun_out/r05/probe2; mkdir -p $o
for L in libtvam_p2 libtvam_p3; do
TVAM_LIB=tools/build/$L.so timeout -k 10 200 python -u tools/proj_ab.py 400 "TVAM_ADJL_NT=768" "TVAM_ADJL_Z=16" > $o/$L.jsonl 2>&1 || exit 1
done
