#!/bin/bash
# r04b: deflate pins (restated Huffman builder, sha golden), then the inflate variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/deflate_sha.py > $OUT/deflate_sha.json 2> $OUT/deflate_sha.err || { tail -20 $OUT/deflate_sha.err; exit 1; }
cat $OUT/deflate_sha.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_bgzf.py -x -v --timeout 250 --timeout-method thread -k "restated" > $OUT/pytest_huff.log 2>&1 || { tail -40 $OUT/pytest_huff.log; exit 1; }
tail -2 $OUT/pytest_huff.log
bash tools/gpu_infl_var.sh $1
