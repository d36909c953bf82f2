#!/bin/bash
# r03 late change check: codec tests, the 20M codec bench, a short e2e bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r03d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_bgzf.py > $OUT/pytest_codec.log 2>&1 || { tail -40 $OUT/pytest_codec.log; exit 1; }
tail -1 $OUT/pytest_codec.log
timeout -k 10 300 python -u tools/bgzf_bench.py 20000000 3 > $OUT/codec_20m.json 2> $OUT/codec_20m.err || { tail -20 $OUT/codec_20m.err; exit 1; }
cat $OUT/codec_20m.json
timeout -k 10 600 python -u bench.py --e2e-only --steps 3 --warmup 1 --no-cpu-baseline --no-realign --no-pcie > $OUT/bench_e2e.json 2> $OUT/bench_e2e.err || { tail -30 $OUT/bench_e2e.err; exit 1; }
grep "e2e:" $OUT/bench_e2e.err | tail -1
