#!/bin/bash
# r03 first pass: the new / changed paths first (deflate + inflate round trips, crafted inflate streams,
# multi-process bootstrap, reference chains with the GPU modules), a short e2e bench, the one-off check
# that the crafted streams break the r02 3941758 literal-batch logic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r03a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bgzf.py tests/test_gpu_inflate.py tests/test_gpu_multiproc.py tests/test_gpu_integration.py > $OUT/pytest_new.log 2>&1 || { tail -60 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
timeout -k 10 300 python -u tools/bgzf_bench.py 20000000 3 > $OUT/codec_20m.json 2> $OUT/codec_20m.err || { tail -20 $OUT/codec_20m.err; exit 1; }
cat $OUT/codec_20m.json
timeout -k 10 600 python -u bench.py --e2e-only --steps 3 --warmup 1 > $OUT/bench_e2e.json 2> $OUT/bench_e2e.err || { tail -30 $OUT/bench_e2e.err; exit 1; }
cut -c1-1200 $OUT/bench_e2e.json
timeout -k 10 120 python -u tools/exp_infl_guard.py > $OUT/exp_guard.log 2>&1; tail -3 $OUT/exp_guard.log
