#!/bin/bash
# r04f: codec tests on the current inflate, then inflate stage times at 20M reads (current vs _var variants)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_bgzf.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest_codec.log 2>&1 || { tail -40 $OUT/pytest_codec.log; exit 1; }
tail -2 $OUT/pytest_codec.log
bash tools/gpu_infl_var.sh $1
