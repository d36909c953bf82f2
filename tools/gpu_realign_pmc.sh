# realign scan kernels: rocprofv3 kernel-trace stats, then SQ instruction counters (separate pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-rlpmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --realign-only > $OUT/bench_rl.json 2> $OUT/bench_rl.err || { tail -20 $OUT/bench_rl.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "k_planes|k_scan_bp|k_realign_scan" -d $OUT/sq -o run --output-format csv -- python3 bench.py --realign-only > $OUT/sq.json 2> $OUT/sq.err || { tail -20 $OUT/sq.err; exit 1; }
python3 - <<'PY' $OUT
import csv, sys, json
d = sys.argv[1]
rows = list(csv.DictReader(open(d + "/prof/run_kernel_stats.csv")))
for r in rows[:12]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f}")
agg = {}
for r in csv.DictReader(open(d + "/sq/run_counter_collection.csv")):
    agg.setdefault(r["Kernel_Name"][:40], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, {c: sum(x) / len(x) for c, x in v.items()})
PY
