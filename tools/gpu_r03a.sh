#!/bin/bash
# r03 first pass: the new GPU tests first (multi-process bootstrap, -R integration, crafted inflate
# streams), then the whole -m gpu suite, then the one-off check that the crafted streams break the
# r02 3941758 literal-batch logic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r03a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bgzf.py tests/test_gpu_multiproc.py tests/test_gpu_integration.py "tests/test_gpu_inflate.py::test_long_codes_before_direct_literal_runs" > $OUT/pytest_new.log 2>&1 || { tail -60 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
timeout -k 10 120 python -u tools/exp_infl_guard.py > $OUT/exp_guard.log 2>&1; cat $OUT/exp_guard.log | tail -5
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
