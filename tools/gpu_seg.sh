#!/bin/bash
# r03 segment inflate: codec tests first, then the 20M codec bench (both inflate implementations)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-seg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_bgzf.py > $OUT/pytest_codec.log 2>&1 || { tail -40 $OUT/pytest_codec.log; exit 1; }
tail -2 $OUT/pytest_codec.log
timeout -k 10 300 python -u tools/bgzf_bench.py 20000000 3 > $OUT/codec_20m.json 2> $OUT/codec_20m.err || { tail -20 $OUT/codec_20m.err; exit 1; }
cat $OUT/codec_20m.json
