#!/bin/bash
# dedup/sort iteration: the GPU parity tests named in $TESTS (default: the sort/dedup suites), then
# the 300M-read kernel-only step with the windowed group stages on and off (A/B)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-kstep}
mkdir -p $OUT
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_pipeline.py tests/test_gpu_dist.py tests/test_gpu_chunked.py"}
timeout -k 10 600 python -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --kernel-only --kernel-steps 3 > $OUT/kstep_win.json 2> $OUT/kstep_win.err || { tail -20 $OUT/kstep_win.err; exit 1; }
cat $OUT/kstep_win.json
OGE_MD_WINDOW=0 timeout -k 10 300 python -u bench.py --kernel-only --kernel-steps 3 > $OUT/kstep_sort.json 2> $OUT/kstep_sort.err || { tail -20 $OUT/kstep_sort.err; exit 1; }
cat $OUT/kstep_sort.json
