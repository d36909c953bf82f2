#!/bin/bash
# r04: the multi-rank tests (world 2/3/4/8 processes on one GPU, piles at G = 4/8), then the whole suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_dist.py -x -v --timeout 500 --timeout-method thread > $OUT/pytest_dist.log 2>&1 || { tail -80 $OUT/pytest_dist.log; exit 1; }
tail -3 $OUT/pytest_dist.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --deselect tests/test_gpu_multiproc.py --deselect tests/test_gpu_dist.py > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
