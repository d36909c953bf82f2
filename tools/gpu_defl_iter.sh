#!/bin/bash
# deflate iteration: BGZF tests, then the codec bench per payload chunk size (OGE_DEFL_CHUNK)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r02i}
READS=${2:-150000000}
CHUNKS=${3:-"2048 4096 8192"}
mkdir -p $OUT
export TMPDIR=/tmp
for c in $CHUNKS; do
  OGE_DEFL_CHUNK=$c timeout -k 10 400 python -u -m pytest tests/test_gpu_bgzf.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_k$c.log 2>&1 || { tail -30 $OUT/pytest_k$c.log; exit 1; }
  echo "chunk=$c $(tail -1 $OUT/pytest_k$c.log)"
done
for c in $CHUNKS; do
  OGE_DEFL_CHUNK=$c timeout -k 10 300 python -u tools/bgzf_bench.py $READS 2 > $OUT/codec_k$c.json 2> $OUT/codec_k$c.err || { tail -20 $OUT/codec_k$c.err; exit 1; }
  echo "chunk=$c $(python3 -c "import json;d=json.load(open('$OUT/codec_k$c.json'));print('deflate', d['ms'], d['GBps'], 'ratio', d['ratio'], 'inflate', d['inflate_ms'])")"
done
