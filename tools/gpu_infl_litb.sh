#!/bin/bash
# inflate literal batching: the inflate tests with OGE_INFL_LITB=4, then the 300M e2e-only bench per setting
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-infl_litb}
mkdir -p $OUT
export TMPDIR=/tmp
OGE_INFL_LITB=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_bgzf.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for B in ${LITBS:-1 4 2}; do
  OGE_INFL_LITB=$B timeout -k 10 400 python -u bench.py --e2e-only --steps 2 --warmup 1 > $OUT/b$B.json 2> $OUT/b$B.err || { tail -20 $OUT/b$B.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b$B.json')); print('litb $B', d['ms_per_step'], d['value'], d['stages_ms']['bgzf_inflate'], d['stages_ms']['bgzf_deflate'])"
done
