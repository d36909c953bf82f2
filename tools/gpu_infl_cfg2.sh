#!/bin/bash
# phase-1 table-size configurations: the inflate tests under each, then the 300M e2e-only bench per cfg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-infl_cfg3}
mkdir -p $OUT
export TMPDIR=/tmp
for C in ${CFGS:-7 8}; do
  OGE_INFL_CFG=$C timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_cfg$C.log 2>&1 || { tail -30 $OUT/pytest_cfg$C.log; exit 1; }
  echo "cfg $C: $(tail -1 $OUT/pytest_cfg$C.log)"
done
for C in ${CFGS:-7 8} 0; do
  OGE_INFL_CFG=$C timeout -k 10 400 python -u bench.py --e2e-only --steps 2 --warmup 1 > $OUT/cfg$C.json 2> $OUT/cfg$C.err || { tail -20 $OUT/cfg$C.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/cfg$C.json')); print('cfg $C', d['ms_per_step'], d['value'], d['stages_ms']['bgzf_inflate'], d['stages_ms']['bgzf_deflate'])"
done
