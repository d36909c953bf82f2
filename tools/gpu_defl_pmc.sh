#!/bin/bash
# BGZF deflate: SQ counters of the k_defl_* kernels (two passes) + kernel stats on a 2M-read stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${PMC_TAG:-r02}/deflpmc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/ks -o run --output-format csv -- python3 tools/bgzf_bench.py 2000000 2 > $OUT/ks.json 2> $OUT/ks.err || { tail -20 $OUT/ks.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --kernel-include-regex "k_defl" -d $OUT/p1 -o run --output-format csv -- python3 tools/bgzf_bench.py 2000000 1 > $OUT/p1.json 2> $OUT/p1.err || { tail -20 $OUT/p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES --kernel-include-regex "k_defl" -d $OUT/p2 -o run --output-format csv -- python3 tools/bgzf_bench.py 2000000 1 > $OUT/p2.json 2> $OUT/p2.err || { tail -20 $OUT/p2.err; exit 1; }
python3 - <<'PY' $OUT
import csv, sys, glob
d = sys.argv[1]
agg = {}
for p in ("p1", "p2"):
    for f in glob.glob(d + "/" + p + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg.setdefault(r["Kernel_Name"][:40], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
for f in glob.glob(d + "/ks/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "defl" in r["Name"] or "infl" in r["Name"]:
            print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
