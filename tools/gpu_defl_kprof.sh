#!/bin/bash
# rocprofv3 kernel stats of the 20M-read deflate (tools/diag_defl.py): the default library, then each VARS library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-defl_kprof}
mkdir -p $OUT
export TMPDIR=/tmp
for v in default ${VARS}; do
  n=$(basename $v .so); a=""; [ "$v" != default ] && a=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run --output-format csv -- python3 tools/diag_defl.py $a > $OUT/$n.txt 2>&1 || { tail -20 $OUT/$n.txt; exit 1; }
  grep "deflate ms" $OUT/$n.txt
  python3 -c "
import csv,glob
f=glob.glob('$OUT/$n/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'defl' in r['Name']: print('  ', r['Name'].split('(')[0][-20:], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg')"
done
