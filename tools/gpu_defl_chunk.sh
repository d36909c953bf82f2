#!/bin/bash
# deflate chunk size (payloads per launch) in the 300M e2e-only bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-defl_chunk}
mkdir -p $OUT
export TMPDIR=/tmp
for K in ${KS:-8192 4096 16384}; do
  OGE_DEFL_CHUNK=$K timeout -k 10 400 python -u bench.py --e2e-only --steps 2 --warmup 1 > $OUT/k$K.json 2> $OUT/k$K.err || { tail -20 $OUT/k$K.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/k$K.json')); print('chunk $K', d['ms_per_step'], d['value'], d['stages_ms']['bgzf_inflate'], d['stages_ms']['bgzf_deflate'])"
done
