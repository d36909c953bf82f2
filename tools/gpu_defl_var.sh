#!/bin/bash
# deflate stage at 20M reads: the default library, then each library variant given (VARS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-defl_var}
mkdir -p $OUT
export TMPDIR=/tmp
for v in default ${VARS}; do
  n=$(basename $v .so); a=""; [ "$v" != default ] && a=$v
  timeout -k 10 200 python -u tools/diag_defl.py $a > $OUT/$n.txt 2>&1 || { tail -20 $OUT/$n.txt; exit 1; }
  grep "deflate ms" $OUT/$n.txt
done
