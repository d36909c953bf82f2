#!/bin/bash
# kernel stats of the codec bench (deflate + inflate) at READS reads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r02n}
READS=${2:-150000000}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ks -o run --output-format csv -- python3 tools/bgzf_bench.py $READS 2 > $OUT/codec.json 2> $OUT/codec.err || { tail -20 $OUT/codec.err; exit 1; }
python3 - <<'PY' $OUT
import csv, glob, sys
d = sys.argv[1]
for f in glob.glob(d + "/ks/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-60s %6s %10.3f ms avg %10.1f ms total" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
