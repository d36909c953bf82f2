# inflate kernel: SQ instruction / wait counters (one pass), on a 4M-read stream
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-inflpmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --kernel-include-regex "k_inflate" -d $OUT/sq -o run --output-format csv -- python3 tools/bgzf_bench.py 4000000 1 > $OUT/sq.json 2> $OUT/sq.err || { tail -20 $OUT/sq.err; exit 1; }
python3 - <<'PY' $OUT
import csv, sys
d = sys.argv[1]
agg = {}
for r in csv.DictReader(open(d + "/sq/run_counter_collection.csv")):
    agg.setdefault(r["Kernel_Name"][:30], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, {c: sum(x) / len(x) for c, x in v.items()})
PY
