#!/bin/bash
# codec iteration: codec tests, 20M deflate/inflate bench, 300M e2e-only bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-codec_iter}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_bgzf.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/bgzf_bench.py 20000000 3 > $OUT/codec20m.json 2> $OUT/codec20m.err || { tail -20 $OUT/codec20m.err; exit 1; }
cut -c1-300 $OUT/codec20m.json
timeout -k 10 400 python -u bench.py --e2e-only --steps 2 --warmup 1 > $OUT/e2e.json 2> $OUT/e2e.err || { tail -20 $OUT/e2e.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/e2e.json')); print('e2e', d['ms_per_step'], d['value'], d['stages_ms']['bgzf_inflate'], d['stages_ms']['bgzf_deflate'])"
