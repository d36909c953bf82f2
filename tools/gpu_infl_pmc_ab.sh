#!/bin/bash
# phase-1 inflate SQ counters per OGE_INFL_CFG on a 20M-read stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r02j}
mkdir -p $OUT
export TMPDIR=/tmp
for c in ${2:-1 3}; do
  OGE_INFL_CFG=$c timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH --kernel-include-regex "k_infl" -d $OUT/c$c -o run --output-format csv -- python3 tools/bgzf_bench.py 20000000 1 > $OUT/c$c.json 2> $OUT/c$c.err || { tail -20 $OUT/c$c.err; exit 1; }
done
python3 - <<'PY' $OUT
import csv, sys, glob
d = sys.argv[1]
for f in sorted(glob.glob(d + "/c*/**/*counter_collection.csv", recursive=True)):
    agg = {}
    for r in csv.DictReader(open(f)):
        agg.setdefault(r["Kernel_Name"][:60], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f.split('/')[2], k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
