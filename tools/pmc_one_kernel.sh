# Counters of one kernel (name regex) in one BASELINE config's bench iteration, summarised on the box
# (per-dispatch averages; raw CSVs deleted).  usage: tools/pmc_one_kernel.sh OUT CONFIG N REGEX
set -euo pipefail
out="$1"; c="$2"; n="$3"; rx="$4"
export TMPDIR=/tmp
mkdir -p "$out"
cmd=(python3 bench.py --config "$c" --n "$n" --steps 1 --warmup 0 --prewarm 0 --cpu-baseline off --breakdown 0)
sets=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $set --kernel-include-regex "$rx" -d "$out/p$i" -o p --output-format csv -- "${cmd[@]}" > "$out/p$i.log" 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$rx" -d "$out/trace" -o k --output-format csv -- "${cmd[@]}" > "$out/trace.log" 2>&1
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        acc[c].append(v)
with open(f"{out}/summary.txt", "w") as fo:
    for c, v in sorted(acc.items()):
        fo.write(f"{c} {sum(v) / len(v):.6g} over {len(v)} dispatches\n")
    for f in glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True):
        fo.write(open(f).read())
PY
find "$out" -name '*.csv' -delete
