#!/bin/bash
# the whole -m gpu suite and smoke (what the driver runs at round end)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
