#!/bin/bash
# deflate A/B over OGE_DEFL_PAD (tokens LDS layout): BGZF + pipeline tests, codec bench at READS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r02o}
READS=${2:-150000000}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bgzf.py tests/test_gpu_pipeline.py tests/test_gpu_inflate.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for p in 1 0; do
  OGE_DEFL_PAD=$p timeout -k 10 300 python -u tools/bgzf_bench.py $READS 2 > $OUT/codec_p$p.json 2> $OUT/codec_p$p.err || { tail -20 $OUT/codec_p$p.err; exit 1; }
  echo "pad=$p $(python3 -c "import json;d=json.load(open('$OUT/codec_p$p.json'));print('deflate', d['ms'], d['GBps'], 'ratio', d['ratio'], 'inflate', d['inflate_ms'])")"
done
