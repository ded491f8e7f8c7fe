# round 5: where the wide kernel's HBM writes come from -- capacity write-backs (NORMAL_WRITEBACK)
# or write-back operations (ALL_TC_OP_WB_WRITEBACK), one --pmc pass each, sliced C4 and rotated C2
set -o pipefail
OUT=${OUT:-gpurun_out/r05w}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
C4="--utts-per-gpu 8 --steps 2 --warmup 1 --cpu-seconds 0 --no-timing"
C2="--steps 2 --warmup 1 --cpu-seconds 0 --no-timing"
run() {  # name, kernel regex, counters, bench args
  timeout -s KILL 120 rocprofv3 --pmc $3 --kernel-include-regex "$2" -d $OUT/$1 -o $1 --output-format csv -- \
    python3 bench.py $4 > $OUT/$1.log 2>&1 || { echo "pmc $1 failed rc=$?"; exit 1; }
}
run c4_write k_persist_wide "WRITE_SIZE" "$C4"
run c4_wb k_persist_wide "TCC_NORMAL_WRITEBACK_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_EA0_WRREQ_sum" "$C4"
run b10_write k_persist_wide "WRITE_SIZE" "--utts-per-gpu 8 --bits 10 --target 3000 --overlap 1500 --steps 2 --warmup 1 --cpu-seconds 0 --no-timing"
run c2_wb "k_persist[^_]" "TCC_NORMAL_WRITEBACK_sum TCC_ALL_TC_OP_WB_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_EA0_WRREQ_sum" "$C2"
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)):
    tot = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        tot[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
    print(f.split('/')[-1], {k: (round(v / 1e6, 2), n[k]) for k, v in tot.items()}, '(millions, dispatch-counter rows)')
PY
