#!/bin/bash
# inflate iteration: correctness tests, then the codec bench for each phase-1 config (OGE_INFL_CFG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r02g}
READS=${2:-150000000}
CFGS=${3:-"0 1 2"}
mkdir -p $OUT
export TMPDIR=/tmp
for c in $CFGS; do
  OGE_INFL_CFG=$c timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_c$c.log 2>&1 || { tail -30 $OUT/pytest_c$c.log; exit 1; }
  echo "cfg=$c $(tail -1 $OUT/pytest_c$c.log)"
done
for c in $CFGS; do
  OGE_INFL_CFG=$c timeout -k 10 300 python -u tools/bgzf_bench.py $READS 2 > $OUT/codec_c$c.json 2> $OUT/codec_c$c.err || { tail -20 $OUT/codec_c$c.err; exit 1; }
  echo "cfg=$c $(python3 -c "import json;d=json.load(open('$OUT/codec_c$c.json'));print(d['inflate_ms'], d['inflate_GBps'], d['ms'])")"
done
