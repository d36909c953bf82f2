#!/bin/bash
# e2e-only bench (300M) under OGE_INFL_CFG settings: which phase-1 configuration is fastest in the chain
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-infl_cfg}
mkdir -p $OUT
export TMPDIR=/tmp
for C in ${CFGS:-1 0 3}; do
  OGE_INFL_CFG=$C timeout -k 10 400 python -u bench.py --e2e-only --steps 2 --warmup 1 > $OUT/cfg$C.json 2> $OUT/cfg$C.err || { tail -20 $OUT/cfg$C.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/cfg$C.json')); print('cfg $C', d['ms_per_step'], d['stages_ms']['bgzf_inflate'], d['stages_ms']['bgzf_deflate'])"
done
