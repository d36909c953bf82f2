#!/bin/bash
# inflate stage at 20M reads: the default library, then each openge_amd/_var/lib_*.so variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-infl_var}
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$NODEFAULT" ] || { timeout -k 10 200 python -u tools/diag_infl.py > $OUT/default.txt 2>&1 || { tail -20 $OUT/default.txt; exit 1; }; }
[ -n "$NODEFAULT" ] || cat $OUT/default.txt
for v in ${VARS-openge_amd/_var/lib_*.so}; do
  n=$(basename $v .so)
  timeout -k 10 200 python -u tools/diag_infl.py $v > $OUT/$n.txt 2>&1 || { tail -20 $OUT/$n.txt; exit 1; }
  cat $OUT/$n.txt
done
