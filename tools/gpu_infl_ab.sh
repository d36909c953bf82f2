#!/bin/bash
# inflate A/B on one box: the codec tests, then the inflate stage at 20M and 100M reads with and without an
# env switch (default OGE_INFL_PREP=0 vs 1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-infl_ab}
VAR=${AB_VAR:-OGE_INFL_PREP}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_bgzf.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
for r in ${AB_READS:-20000000 100000000}; do
  for v in 0 1; do
    env $VAR=$v DIAG_READS=$r timeout -k 10 200 python -u tools/diag_infl.py > $OUT/r${r}_$v.txt 2>&1 || { tail -20 $OUT/r${r}_$v.txt; exit 1; }
    echo "$VAR=$v $(grep reads $OUT/r${r}_$v.txt)"
  done
done
