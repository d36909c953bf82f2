#!/bin/bash
# literal batches after matches (OGE_DEFL_AFTER / OGE_INFL_AFTER): codec tests under both, 20M deflate
# A/B, 300M e2e-only A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-after}
mkdir -p $OUT
export TMPDIR=/tmp
OGE_DEFL_AFTER=1 OGE_INFL_AFTER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_bgzf.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for A in 0 1; do
  OGE_DEFL_AFTER=$A timeout -k 10 300 python -u tools/bgzf_bench.py 20000000 3 > $OUT/defl$A.json 2> $OUT/defl$A.err || { tail -20 $OUT/defl$A.err; exit 1; }
  echo "DEFL_AFTER=$A $(cut -c1-260 $OUT/defl$A.json)"
done
for A in 1 0; do
  OGE_DEFL_AFTER=$A OGE_INFL_AFTER=$A timeout -k 10 400 python -u bench.py --e2e-only --steps 2 --warmup 1 > $OUT/e2e$A.json 2> $OUT/e2e$A.err || { tail -20 $OUT/e2e$A.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/e2e$A.json')); print('after $A', d['ms_per_step'], d['value'], d['stages_ms']['bgzf_inflate'], d['stages_ms']['bgzf_deflate'])"
done
